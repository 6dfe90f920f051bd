"""Per-wave duration distribution of hwy_step_kernel (development aid; needs make prof).
probe_waves.py [E] [steps]"""
import ctypes, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "highway-rope-ppo_amd"))
import numpy as np
import torch
import hwy.native as native

native.LIB_PATH = os.environ.get("HWY_PROF_LIB") or os.path.join(os.path.dirname(native.LIB_PATH), "libhwy_waves.so")
from config.base_config import HIGHWAY_CONFIG
from hwy.vec_env import HighwayVecEnv

E = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
S = int(sys.argv[2]) if len(sys.argv) > 2 else 30
env = HighwayVecEnv(HIGHWAY_CONFIG, num_envs=E, device="cuda:0", autoreset=True, seed_base=42)
env.reset()
L = native.lib()
n = 5 * min(E, 16384)
buf = (ctypes.c_ulonglong * n)()
g = torch.Generator(device="cuda:0").manual_seed(0)
recs = []
for t in range(S):
    env.step(torch.rand(E, 2, device="cuda:0", generator=g) * 0.6 - 0.3)
    torch.cuda.synchronize()
    if t < 5:
        continue
    L.hwy_debug_wave_times(buf, n)
    recs.append(np.frombuffer(buf, dtype=np.uint64).reshape(-1, 5).copy())
dur = np.concatenate([(r[:, 1].astype(np.int64) - r[:, 0].astype(np.int64)) for r in recs])
q = np.percentile(dur, [0, 10, 50, 90, 99, 99.9, 100])
print(f"E={E}: wave duration clk  min {q[0]:.0f}  p10 {q[1]:.0f}  p50 {q[2]:.0f}  p90 {q[3]:.0f}  "
      f"p99 {q[4]:.0f}  p99.9 {q[5]:.0f}  max {q[6]:.0f}  mean {dur.mean():.0f}")
for si, r in enumerate(recs[:3] + recs[-1:]):
    st = r[:, 0].astype(np.int64)
    d = r[:, 1].astype(np.int64) - st
    f = r[:, 2]
    done = (f & 1).astype(bool)
    hw = ((f >> 8) & 0xffffffff).astype(np.int64)
    xcc = (f >> 40).astype(np.int64)
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 15
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    cukey = ((xcc * 8 + se) * 2 + sh) * 16 + cu
    simdkey = cukey * 4 + simd
    _, inv_s, cnt_s = np.unique(simdkey, return_inverse=True, return_counts=True)
    _, inv_c, cnt_c = np.unique(cukey, return_inverse=True, return_counts=True)
    wps = cnt_s[inv_s]
    print(f"step sample {si}: xccs {np.unique(xcc).size}, CUs used {cnt_c.size}, SIMDs used {cnt_s.size}; "
          f"waves/CU hist {dict(zip(*np.unique(cnt_c, return_counts=True)))}; waves/SIMD hist "
          f"{dict(zip(*np.unique(cnt_s, return_counts=True)))}")
    for k in np.unique(wps):
        print(f"   waves on SIMD={k}: n={np.sum(wps == k)} mean dur {d[wps == k].mean():.0f} max {d[wps == k].max():.0f}")
    # start offset within each XCC
    for x in np.unique(xcc)[:2]:
        m = xcc == x
        off = st[m] - st[m].min()
        end = st[m] + d[m] - st[m].min()
        print(f"   xcc {x}: start offset p50 {np.median(off):.0f} max {off.max():.0f}; end p10 {np.percentile(end, 10):.0f} "
              f"p50 {np.median(end):.0f} max {end.max():.0f}; corr(start, dur) {np.corrcoef(off, d[m])[0, 1]:.2f}")
    mk = np.zeros(cnt_s.size)
    s0 = np.full(cnt_s.size, np.iinfo(np.int64).max)
    np.minimum.at(s0, inv_s, st)
    np.maximum.at(mk, inv_s, st + d - s0[inv_s])
    qq = np.percentile(mk, [0, 10, 50, 90, 99, 100])
    print("   SIMD makespan (last end - first start) min/p10/p50/p90/p99/max " + " ".join(f"{v:.0f}" for v in qq))
    sk = np.unique(simdkey)
    for name, sel in (("xcc", sk // 4 // 16 // 2 // 8), ("se", (sk // 4 // 16 // 2) % 8), ("sh", (sk // 4 // 16) % 2),
                      ("cu", (sk // 4) % 16), ("simd", sk % 4)):
        print(f"   makespan by {name}: " + " ".join(f"{u}:{mk[sel == u].mean() / 1e3:.0f}k" for u in np.unique(sel)))
    rts, rte = r[:, 3].astype(np.int64), r[:, 4].astype(np.int64)
    x_all = sk // 4 // 16 // 2 // 8
    print("   realtime (100 MHz) per xcc: start-min / end-max rel. to global min start: " +
          " ".join(f"{u}:{(rts[xcc == u].min() - rts.min())}/{(rte[xcc == u].max() - rts.min())}" for u in np.unique(xcc)))
    print("   memtime/realtime tick ratio per xcc: " + " ".join(
          f"{u}:{np.median(d[xcc == u] / np.maximum(rte[xcc == u] - rts[xcc == u], 1)):.1f}" for u in np.unique(xcc)))
    rd = rte - rts
    cls = (np.arange(rd.size) // 4) % 8
    print("   realtime dur by env class (e/4)%8: " + " ".join(f"{u}:{rd[cls == u].mean():.0f}" for u in range(8)) +
          "  | by xcc: " + " ".join(f"{u}:{rd[xcc == u].mean():.0f}" for u in np.unique(xcc)))
    if si > 0:
        print(f"   corr(dur this step, dur prev sample) per env: {np.corrcoef(rd, prev_rd)[0, 1]:.2f}")
    prev_rd = rd
    ss = np.zeros(cnt_s.size); np.maximum.at(ss, inv_s, st - s0[inv_s])
    print(f"   SIMD start spread p50 {np.median(ss):.0f} max {ss.max():.0f}")
    print(f"   done waves mean {d[done].mean() if done.any() else 0:.0f}, live {d[~done].mean():.0f}")
