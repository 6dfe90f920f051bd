"""hwy_step timing for the configs[2]/[4] observation shapes (30 rows, shuffled, PE d 4) through
the reference's make_env (development aid): probe_step_pe.py [pe] [E ...]; HWY_LIB overrides
the library."""
import os, sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "highway-rope-ppo_amd"))
import torch
import hwy.native as native

if os.environ.get("HWY_LIB"):
    native.LIB_PATH = os.environ["HWY_LIB"]
from config.base_config import HIGHWAY_CONFIG
from experiments.config import Condition
from experiments.wrappers import make_env

pe = sys.argv[1] if len(sys.argv) > 1 else "rope"
cond = {"none": Condition.SHUFFLED, "rope": Condition.SHUFFLED_ROPE,
        "dist": Condition.SHUFFLED_DISTPE, "rank": Condition.SHUFFLED_RANKPE}[pe]
dev = torch.device("cuda", 0)
for E in [int(x) for x in (sys.argv[2:] or ["16384"])]:
    env = make_env(cond, HIGHWAY_CONFIG, d_embed=4 if pe != "none" else None,
                   env_overrides={"observation": {"vehicles_count": 30, "order": "shuffled"},
                                  "num_envs": E, "device": dev, "autoreset": True}).unwrapped
    env.set_seed_schedule(42)
    env.reset()
    N, Fo = env.obs_rows, env.obs_features
    obs = torch.empty(E, N * Fo, device=dev)
    r = torch.empty(E, device=dev)
    te = torch.empty(E, dtype=torch.uint8, device=dev)
    tr = torch.empty(E, dtype=torch.uint8, device=dev)
    er = torch.empty(E, device=dev)
    el = torch.empty(E, dtype=torch.int32, device=dev)
    a = torch.zeros(E, 2, device=dev)
    for _ in range(5):
        env.step_into(a, obs, r, te, tr, er, el)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 50
    s.record()
    for _ in range(n):
        a.uniform_(-0.3, 0.3)
        env.step_into(a, obs, r, te, tr, er, el)
    e.record()
    torch.cuda.synchronize()
    print(f"pe={pe} E={E}: {s.elapsed_time(e) / n:.3f} ms/step", flush=True)
