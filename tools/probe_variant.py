"""hwy_step timing with an alternative build of libhwy (development aid):
probe_variant.py <path/to/lib.so> [E]"""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "highway-rope-ppo_amd"))
import torch
import hwy.native as native

native.LIB_PATH = os.path.abspath(sys.argv[1])
from config.base_config import HIGHWAY_CONFIG
from hwy.vec_env import HighwayVecEnv

E = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
env = HighwayVecEnv(HIGHWAY_CONFIG, num_envs=E, device="cuda:0", autoreset=True, seed_base=42)
env.reset()
g = torch.Generator(device="cuda:0").manual_seed(0)
acts = torch.rand(60, E, 2, device="cuda:0", generator=g) * 0.6 - 0.3
for i in range(10):
    env.step(acts[i])
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for i in range(10, 60):
    env.step(acts[i])
e.record()
torch.cuda.synchronize()
print(f"{os.path.basename(sys.argv[1]):28s} {s.elapsed_time(e) / 50 * 1e3:8.1f} us/step", flush=True)
