"""In-kernel shader clock of ppo_rows_c / ppo_wgrad (clock-probe build, make variant V=clk
VEXTRA=-DHWY_CLOCK_PROBE): s_memtime / s_memrealtime deltas per workgroup after ~2 s of
back-to-back minibatch steps (MI355X_MICROARCH.md, DVFS item 6).  probe_clock.py [rows] [seconds]"""
import ctypes, os, sys, time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "highway-rope-ppo_amd"))
import torch
import hwy.native as native

native.LIB_PATH = os.environ.get("HWY_LIB") or os.path.join(os.path.dirname(native.LIB_PATH), "libhwy_clk.so")
from hwy.ppo_native import FusedPPO
from ppo.agent import PPOAgent

dev = torch.device("cuda", 0)
mb = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
secs = float(sys.argv[2]) if len(sys.argv) > 2 else 2.0
S, H, nmb = 60, 256, 32
torch.manual_seed(0)
ag = PPOAgent(S, 2, lr=3e-4, epochs=1, hidden_dim=H, device=dev, use_graphs=False, backend="hip")
n = mb * nmb
s = torch.randn(n, S, device=dev); z = torch.randn(n, 2, device=dev)
lp = torch.randn(n, device=dev) - 2; adv = torch.randn(n, device=dev); ret = torch.randn(n, device=dev)
perm = torch.randperm(n, device=dev)
F = FusedPPO(ag, mb, nmb, use_graphs=True)
L = native.lib()
L.hwy_ppo_debug_sections.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = (ctypes.c_ulonglong * 16)()
t0 = time.time()
while time.time() - t0 < secs:  # warm the clock governor into its steady state
    F.run(s, z, lp, adv, ret, perm)
torch.cuda.synchronize()
L.hwy_ppo_debug_sections(buf, 1)
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record()
for _ in range(10):
    F.run(s, z, lp, adv, ret, perm)
ev1.record()
torch.cuda.synchronize()
L.hwy_ppo_debug_sections(buf, 1)
print(f"rows={mb}: {ev0.elapsed_time(ev1) / (10 * nmb) * 1e3:.1f} us per minibatch step")
for k, name in ((0, "ppo_rows_c"), (1, "ppo_wgrad")):
    mt, rt = buf[2 * k], buf[2 * k + 1]
    if rt:
        print(f"  {name}: {mt / rt * 100e6 / 1e9:.3f} GHz in-kernel clock "
              f"({mt / rt * 100:.0f} shader cycles per us), workgroup lifetime sum {rt / 100:.0f} us")

# workgroup timeline of the last launch of each kernel: lifetimes, spread, and the two-per-CU
# pairing of ppo_rows_c (HW_ID: CU id bits 8-11, SH 12, SE 13-15; XCC id)
import numpy as np
L.hwy_ppo_debug_wgtimes.argtypes = [ctypes.c_void_p]
wt = (ctypes.c_ulonglong * (2 * 1024 * 3))()
L.hwy_ppo_debug_wgtimes(wt)
a = np.frombuffer(wt, dtype=np.uint64).reshape(2, 1024, 3).astype(np.int64)
rt = 64 if mb >= 64 * 256 else 32  # ppo_rows_c64 / ppo_rows_c tiles at H 256
for k, name, nwg in ((0, "ppo_rows_c", mb // rt), (1, "ppo_wgrad", 269)):
    t = a[k][:nwg]
    t = t[t[:, 1] > 0]
    t0, t1 = t[:, 0].min(), t[:, 1].max()
    life = (t[:, 1] - t[:, 0]) / 100.0
    st = (t[:, 0] - t0) / 100.0
    en = (t[:, 1] - t0) / 100.0
    print(f"  {name}: {len(t)} WGs, span {(t1 - t0) / 100:.1f} us; start max {st.max():.1f} us; "
          f"lifetime mean {life.mean():.1f} min {life.min():.1f} max {life.max():.1f} us; "
          f"end p10/p50/p90 {np.percentile(en, 10):.1f}/{np.percentile(en, 50):.1f}/{np.percentile(en, 90):.1f}")
    cu = (t[:, 2] & 0xffffffff) >> 8 & 0xff
    xcc = t[:, 2] >> 32
    key = xcc * 256 + cu
    if k == 0:
        import collections
        grp = collections.defaultdict(list)
        for i, kk in enumerate(key):
            grp[int(kk)].append(i)
        sizes = collections.Counter(len(v) for v in grp.values())
        print(f"    WGs per CU slot: {dict(sizes)}")
        gaps = [abs(en[v[0]] - en[v[1]]) for v in grp.values() if len(v) == 2]
        if gaps:
            print(f"    end-time gap between a CU's two WGs: mean {np.mean(gaps):.1f} max {np.max(gaps):.1f} us")
    if k == 1:  # balanced partition: id % 8 = slice, id / 8 = j; j < 26 main, then extras
        j = np.arange(nwg)[a[k][:nwg, 1] > 0] // 8
        for lab, m in (("main", j < 26), ("extras", (j >= 26) & (j < 31)), ("last extra (+head sums)", j == 31)):
            if m.any():
                print(f"    {lab:24s} n={m.sum():3d} start {st[m].mean():5.1f} lifetime mean {life[m].mean():5.1f} "
                      f"max {life[m].max():5.1f} end max {en[m].max():5.1f} us")

