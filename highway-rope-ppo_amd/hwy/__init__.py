"""hwy -- MI355X-native vectorised highway-v0 (libhwy.so) and its torch bindings.

    from hwy import HighwayVecEnv, ops
    env = HighwayVecEnv(HIGHWAY_CONFIG, num_envs=4096, device="cuda:0")

Submodules: _abi (ctypes mirror of include/hwy.h), native (library loader), vec_env
(HighwayVecEnv), ops (obs_pe / gae), gym (gymnasium API surface), single_env (E = 1 numpy
facade used by the reference-compatible wrappers).
"""

from ._abi import (  # noqa: F401
    FEATURES,
    HWY_ABI_VERSION,
    PE_DIST,
    PE_NONE,
    PE_RANK,
    PE_ROPE,
    HwyConfig,
    config_from_dict,
)
from .native import HwyNativeError, build  # noqa: F401


def __getattr__(name):
    import importlib

    if name == "HighwayVecEnv":
        return importlib.import_module(".vec_env", __name__).HighwayVecEnv
    if name in ("ops", "vec_env", "single_env", "gym"):
        return importlib.import_module("." + name, __name__)
    raise AttributeError(name)
