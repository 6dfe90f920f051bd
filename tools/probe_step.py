"""Quick timing probe of hwy_step / hwy_reset on one GPU (development aid)."""
import sys, os, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "highway-rope-ppo_amd"))
import torch
import hwy.native as native

if os.environ.get("HWY_LIB"):  # a variant library (development A/B)
    native.LIB_PATH = os.environ["HWY_LIB"]
from config.base_config import HIGHWAY_CONFIG
from hwy.vec_env import GroupEnvStep, HighwayVecEnv

# the product's launch (LockstepRollout): hwy_step_group over this one handle, the launch
# parameters read from a device table; PROBE_SOLO=1 times hwy_step's by-value kernel instead
SOLO = bool(os.environ.get("PROBE_SOLO"))

for E in [int(x) for x in (sys.argv[1:] or ["4096", "16384"])]:
    env = HighwayVecEnv(HIGHWAY_CONFIG, num_envs=E, device="cuda:0", autoreset=True, seed_base=42)
    env.reset()
    a = torch.zeros(E, 2, device="cuda:0")
    io = (a, torch.empty_like(env.obs_buf), torch.empty(E, device="cuda:0"),
          torch.empty(E, dtype=torch.uint8, device="cuda:0"),
          torch.empty(E, dtype=torch.uint8, device="cuda:0"), None, None)
    g = GroupEnvStep([env])

    def step():
        if SOLO:
            env.step_into(*io)
        else:
            g.launch([io])

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 50
    s.record()
    for _ in range(n):
        a.uniform_(-0.3, 0.3)
        step()
    e.record(); torch.cuda.synchronize()
    ms = s.elapsed_time(e) / n
    print(f"E={E}: {ms:.3f} ms/step  -> {E/ms*1e3/1e6:.2f} M env-steps/s", flush=True)
    env.close()
