"""Event counts of a counting build of hwy_step (development aid): probe_counts.py <lib.so> [E]"""
import ctypes, os, sys
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
for i in range(60):
    env.step(torch.rand(E, 2, device="cuda:0", generator=g) * 0.6 - 0.3)
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * 8)()
native.lib().hwy_cnt(buf)
print(list(buf))
