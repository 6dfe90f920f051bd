import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "highway-rope-ppo_amd")
for p in (PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running")


# development A/B only (tools/ab.sh TESTS=1): run the suite against a variant library build
if os.environ.get("HWY_LIB"):
    import hwy.native as _native

    _native.LIB_PATH = os.environ["HWY_LIB"]
