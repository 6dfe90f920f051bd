"""Per-frame HIP-vs-oracle divergence finder (development aid; runs on the GPU box)."""
import sys, os
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "highway-rope-ppo_amd")); sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
from hwy import _abi
from parity_util import make_cfg, policy_actions, FIELD_NAMES
from test_env_parity_gpu import HipEnv
from oracle.oracle import OracleEnv

def fstate(st):
    return {n: (st[i].view(np.float32) if i < 9 else st[i].view(np.int32)) for i, n in enumerate(FIELD_NAMES)}

for order in ["sorted"]:
    cfg = make_cfg(E=48, order=order, policy_frequency=15)
    V = cfg.vehicles_count + 1
    hip, ora = HipEnv(cfg), OracleEnv(cfg)
    hip.reset(); ora.reset()
    rng = np.random.default_rng(1)
    for t in range(400):
        prev = ora.state.copy()
        a = policy_actions(rng, cfg.num_envs, t)
        hip.step(a); ora.step(a)
        sh, so = hip.state(), ora.state
        if not np.array_equal(sh, so):
            idx = np.argwhere(sh != so)
            print(f"frame {t}: {len(idx)} words differ")
            envs = sorted(set(idx[:, 1]))
            for e in envs[:3]:
                vs = sorted(set(idx[idx[:, 1] == e][:, 2]))
                print(f" env {e}: vehicles {vs}")
                P, H, O = fstate(prev), fstate(sh), fstate(so)
                for v in vs[:4]:
                    print(f"  veh {v}: fields {[FIELD_NAMES[f] for f in sorted(set(idx[(idx[:,1]==e)&(idx[:,2]==v)][:,0]))]}")
                    for n in FIELD_NAMES[:12]:
                        print(f"    {n:12s} prev={P[n][e,v]!r:>14} hip={H[n][e,v]!r:>14} ora={O[n][e,v]!r:>14}")
                    dt = np.float32(1/15)
                    print(f"    acc hip={(H['speed'][e,v]-P['speed'][e,v])/dt} ora={(O['speed'][e,v]-P['speed'][e,v])/dt}")
                # neighbourhood
                ln = P['lane'][e, :V]; x = P['x'][e, :V]
                order_ = np.argsort(x)
                print("  env vehicles (idx,x,y,lane,tlane,spd):")
                for k in order_:
                    print(f"    {k:2d} {x[k]:9.3f} {P['y'][e,k]:7.3f} {ln[k]} {P['target_lane'][e,k]} {P['speed'][e,k]:7.3f} tmr={P['timer'][e,k]:.3f} fl={P['flags'][e,k]}")
            break
    else:
        print("no divergence in 400 frames")
    hip.close()
