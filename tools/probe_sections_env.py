"""Which sections make the slow envs slow (development aid; needs make prof).

Per-env section clocks of hwy_step_kernel over `steps` launches: the envs ranked by their total,
then the mean clocks per step of each section for the slowest 1 %, 10 % and the median decile.
The launch ends with its slowest wave, so the sections that grow in the slow envs are the ones
that set the kernel time.  probe_sections_env.py [E] [steps]"""
import ctypes, os, sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "highway-rope-ppo_amd"))
import numpy as np
import torch
import hwy.native as native

native.LIB_PATH = os.environ.get("HWY_PROF_LIB") or os.path.join(os.path.dirname(native.LIB_PATH), "libhwy_prof.so")
from config.base_config import HIGHWAY_CONFIG
from hwy.vec_env import HighwayVecEnv

NS = 18
NAMES = {15: "load", 0: "frame head", 9: "road order (frame 0)", 1: "neighbours", 2: "gathers+self_a",
         3: "MOBIL", 4: "abort check", 5: "target IDM+steering", 6: "kinematics",
         7: "post-move order", 10: "collision candidates", 8: "pre-check+SAT", 11: "reward",
         12: "reset", 13: "observe", 14: "store (env words)", 16: "frames exit", 17: "store (vehicles)"}
E = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1
env = HighwayVecEnv(HIGHWAY_CONFIG, num_envs=E, device="cuda:0", autoreset=True, seed_base=42)
env.reset()
a = torch.zeros(E, 2, device="cuda:0")
L = native.lib()
L.hwy_debug_sections.argtypes = [ctypes.c_void_p, ctypes.c_int]
L.hwy_debug_sections_env.argtypes = [ctypes.c_void_p, ctypes.c_int]
tot = (ctypes.c_ulonglong * NS)()
for _ in range(5):
    env.step(a)
torch.cuda.synchronize()
L.hwy_debug_sections(tot, 1)
g = torch.Generator(device="cuda:0").manual_seed(0)
per = np.zeros((E, NS))
for _ in range(n):
    a.copy_(torch.rand(E, 2, device="cuda:0", generator=g) * 0.6 - 0.3)
    env.step(a)
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * (NS * E))()
    L.hwy_debug_sections_env(buf, E)
    L.hwy_debug_sections(tot, 1)
    step = np.frombuffer(buf, dtype=np.uint64).reshape(E, NS).astype(np.float64)
    per += step / n
    t = step.sum(1)
    order = np.argsort(t)
    print(f"step: env clocks min {t.min():.0f} p50 {np.median(t):.0f} p99 {np.percentile(t, 99):.0f} "
          f"max {t.max():.0f}; slowest envs {order[-5:][::-1].tolist()}")
t = per.sum(1)
order = np.argsort(t)
groups = {"slowest 1%": order[-max(1, E // 100):], "slowest 10%": order[-E // 10:],
          "median decile": order[int(0.45 * E):int(0.55 * E)], "fastest 10%": order[:E // 10]}
print(f"E={E}, {n} step(s); mean clocks per env-step by section:")
print(f"  {'section':24s}" + "".join(f"{k:>15s}" for k in groups))
for i in sorted(NAMES, key=lambda i: -per[groups['slowest 1%'], i].mean()):
    print(f"  {NAMES[i]:24s}" + "".join(f"{per[g, i].mean():15,.0f}" for g in groups.values()))
print(f"  {'total':24s}" + "".join(f"{t[g].mean():15,.0f}" for g in groups.values()))
