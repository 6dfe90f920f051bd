"""hwy_step time vs frames per step (sim_freq / policy_freq): per-frame cost and fixed cost
(development aid)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "highway-rope-ppo_amd"))
import torch
from config.base_config import HIGHWAY_CONFIG
from hwy.vec_env import HighwayVecEnv

E = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
for fr in (1, 2, 4, 8, 15):
    cfg = dict(HIGHWAY_CONFIG, simulation_frequency=fr, policy_frequency=1)
    env = HighwayVecEnv(cfg, num_envs=E, device="cuda:0", autoreset=True, seed_base=42)
    env.reset()
    a = torch.zeros(E, 2, device="cuda:0")
    for _ in range(5):
        env.step(a)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 50
    s.record()
    for _ in range(n):
        env.step(a)
    e.record()
    torch.cuda.synchronize()
    print(f"frames={fr:2d}: {s.elapsed_time(e) / n * 1e3:8.1f} us/step", flush=True)
    env.close()
