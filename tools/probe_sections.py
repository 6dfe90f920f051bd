"""Per-section shader-clock breakdown of hwy_step_kernel (development aid).

Needs the profiling build: make -C highway-rope-ppo_amd/csrc prof  (-> hwy/libhwy_prof.so).
"""
import ctypes, os, sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "highway-rope-ppo_amd"))
import torch
import hwy.native as native

native.LIB_PATH = os.environ.get("HWY_PROF_LIB") or os.path.join(os.path.dirname(native.LIB_PATH), "libhwy_prof.so")
from config.base_config import HIGHWAY_CONFIG
from hwy.vec_env import HighwayVecEnv

NAMES = {15: "load", 0: "frame head", 9: "road order (frame 0)", 1: "neighbours", 2: "gathers+self_a",
         3: "MOBIL", 4: "abort check", 5: "target IDM+steering", 6: "kinematics",
         7: "post-move order", 10: "collision candidates", 8: "pre-check+SAT", 11: "reward",
         12: "reset", 13: "observe",
         14: "store (env words)", 16: "frames exit", 17: "store (vehicles)"}
E = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
env = HighwayVecEnv(HIGHWAY_CONFIG, num_envs=E, device="cuda:0", autoreset=True, seed_base=42)
env.reset()
a = torch.zeros(E, 2, device="cuda:0")
L = native.lib()
L.hwy_debug_sections.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = (ctypes.c_ulonglong * 18)()
for _ in range(5):
    env.step(a)
torch.cuda.synchronize()
L.hwy_debug_sections(buf, 1)
n = 40
for _ in range(n):
    a.uniform_(-0.3, 0.3)
    env.step(a)
torch.cuda.synchronize()
L.hwy_debug_sections(buf, 1)
tot = sum(buf)
print(f"E={E}, {n} steps; clocks per wave-step by section:")
for i in sorted(NAMES, key=lambda i: -buf[i]):
    print(f"  {NAMES[i]:24s} {buf[i] / (E * n):12,.0f}  {100 * buf[i] / tot:5.1f}%")
print(f"  {'total':24s} {tot / (E * n):12,.0f}")
