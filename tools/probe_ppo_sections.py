"""Per-phase shader-clock breakdown of ppo_rows / ppo_wgrad (development aid):
probe_ppo_sections.py [H] [minibatch rows]; HWY_ROWS_RT=16|32 forces ppo_rows' row tile.

Needs the profiling build: make -C highway-rope-ppo_amd/csrc prof  (-> hwy/libhwy_prof.so).
"""
import ctypes, os, sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "highway-rope-ppo_amd"))
import torch
import hwy.native as native

native.LIB_PATH = os.environ.get("HWY_PROF_LIB") or os.path.join(os.path.dirname(native.LIB_PATH), "libhwy_prof.so")
from hwy.ppo_native import FusedPPO
from ppo.agent import PPOAgent

dev = torch.device("cuda", 0)
S, H, nmb = 60, int(sys.argv[1]) if len(sys.argv) > 1 else 256, 32
mb = int(sys.argv[2]) if len(sys.argv) > 2 else 4096  # minibatch rows
torch.manual_seed(0)
ag = PPOAgent(S, 2, lr=3e-4, epochs=1, hidden_dim=H, device=dev, use_graphs=False, backend="hip")
n = mb * nmb
s = torch.randn(n, S, device=dev)
z = torch.randn(n, 2, device=dev)
lp = torch.randn(n, device=dev) - 2
adv = torch.randn(n, device=dev)
ret = torch.randn(n, device=dev)
perm = torch.randperm(n, device=dev)
F = FusedPPO(ag, mb, nmb, use_graphs=True)
L = native.lib()
L.hwy_ppo_debug_sections.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = (ctypes.c_ulonglong * 16)()
F.run(s, z, lp, adv, ret, perm)
torch.cuda.synchronize()
L.hwy_ppo_debug_sections(buf, 1)
reps = 5
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record()
for _ in range(reps):
    F.run(s, z, lp, adv, ret, perm)
ev1.record()
torch.cuda.synchronize()
L.hwy_ppo_debug_sections(buf, 1)
steps = reps * nmb
print(f"H={H}: {ev0.elapsed_time(ev1) / steps * 1e3:.1f} us per minibatch step (graph, incl. adam)")
rt = int(os.environ.get("HWY_ROWS_RT", "0")) or (
    64 if H == 256 and mb >= 64 * 256 else (32 if H <= 256 and mb >= 8192 else 16))
n1 = (mb + rt - 1) // rt  # ppo_rows workgroups (rows_tile in ppo_kernels.hip)
print(f"  ppo_rows: {rt} rows per workgroup, {n1} workgroups")
names = {0: "rows: gather", 1: "rows: h1", 2: "rows: h2", 3: "rows: ac", 7: "rows: head sums",
         11: "rows: head rows", 4: "rows: head sync", 5: "rows: dh2", 6: "rows: dh1"}
tot = sum(buf[i] for i in names)
for i, nm in names.items():
    print(f"  {nm:22s} {buf[i] / (steps * n1):10,.0f} clk/WG  {100 * buf[i] / tot:5.1f}%")
tm, tn = (H + 127) // 128, (H + 63) // 64  # 128x64 ppo_wgrad tiles
ntile = ((2 * H + 127) // 128) * tn + tm * tn + tm * ((S + 63) // 64)
split = max(1, min(8, 256 // ntile, (mb + 63) // 64))
nh = (3 * H + 9 + 63) // 64
print(f"  wgrad tiles={ntile} split={split} head WGs={nh}")
print(f"  {'wgrad: chunk loop':22s} {buf[8] / (steps * ntile * split):10,.0f} clk/WG")
print(f"  {'wgrad: slab write':22s} {buf[9] / (steps * ntile * split):10,.0f} clk/WG")
print(f"  {'wgrad: head WG':22s} {buf[10] / (steps * nh):10,.0f} clk/WG")
