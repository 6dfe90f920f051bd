"""HIP env step/reset vs the CPU oracle, bit for bit (state words, observations, rewards, flags).

The oracle (oracle/hwy_oracle.c) runs upstream highway-env's algorithm sequentially, vehicle
by vehicle; the kernel runs one wavefront per env.  Both use hwy_math.h, so every word must be
identical: any difference is a bug in the parallel formulation.
"""

import numpy as np
import pytest
import torch

from hwy import _abi
from hwy.native import check, lib, ptr
from oracle.oracle import OracleEnv
from parity_util import diff_state, make_cfg, pe_table_for, policy_actions

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


class HipEnv:
    """Direct C-ABI driver (no Python env layer) so the test exercises exactly libhwy.so."""

    def __init__(self, cfg, table=None):
        import ctypes

        self.cfg = cfg
        self.E, self.N, self.Fo = cfg.num_envs, cfg.obs_vehicles, cfg.obs_features()
        self.h = ctypes.c_void_p()
        check(lib().hwy_create(ctypes.byref(cfg), 0, ctypes.byref(self.h)), "hwy_create")
        if table is not None:
            t = np.ascontiguousarray(table, np.float32)
            check(lib().hwy_set_pe_table(self.h, t.ctypes.data_as(ctypes.c_void_p), t.size),
                  "hwy_set_pe_table")
        self.obs = torch.zeros(self.E, self.N, self.Fo, device=DEV)
        self.rew = torch.zeros(self.E, device=DEV)
        self.term = torch.zeros(self.E, dtype=torch.uint8, device=DEV)
        self.trunc = torch.zeros(self.E, dtype=torch.uint8, device=DEV)
        self.er = torch.zeros(self.E, device=DEV)
        self.el = torch.zeros(self.E, dtype=torch.int32, device=DEV)

    def reset(self, seeds=None):
        s = None if seeds is None else torch.as_tensor(seeds.astype(np.int64), device=DEV)
        check(lib().hwy_reset(self.h, ptr(s), None, ptr(self.obs), None), "hwy_reset")
        torch.cuda.synchronize()
        return self.obs.cpu().numpy()

    def step(self, a):
        at = torch.as_tensor(a, device=DEV).contiguous()
        check(lib().hwy_step(self.h, ptr(at), ptr(self.obs), ptr(self.rew), ptr(self.term),
                             ptr(self.trunc), ptr(self.er), ptr(self.el), None), "hwy_step")
        torch.cuda.synchronize()
        return (self.obs.cpu().numpy(), self.rew.cpu().numpy(), self.term.cpu().numpy(),
                self.trunc.cpu().numpy(), self.er.cpu().numpy(), self.el.cpu().numpy())

    def state(self):
        out = torch.zeros(_abi.NFIELDS, self.E, 64, dtype=torch.int32, device=DEV)
        check(lib().hwy_export_state(self.h, ptr(out), None), "export")
        torch.cuda.synchronize()
        return out.cpu().numpy().view(np.uint32)

    def set_state(self, st):
        t = torch.as_tensor(np.ascontiguousarray(st).view(np.int32), device=DEV)
        check(lib().hwy_import_state(self.h, ptr(t), None), "import")
        torch.cuda.synchronize()

    def close(self):
        lib().hwy_destroy(self.h)


def run_parity(cfg, steps, table=None, seed=0, action_fn=policy_actions):
    hip = HipEnv(cfg, table)
    ora = OracleEnv(cfg, table)
    V = cfg.vehicles_count + 1
    try:
        o_h = hip.reset()
        o_o = ora.reset()
        d = diff_state(hip.state(), ora.state, V)
        assert d is None, f"reset state: {d}"
        np.testing.assert_array_equal(o_h, o_o, err_msg="reset obs")
        rng = np.random.default_rng(seed)
        stats = dict(crashes=0, dones=0, lane_changes=0)
        for t in range(steps):
            a = action_fn(rng, cfg.num_envs, t)
            rh = hip.step(a)
            ro = ora.step(a)
            d = diff_state(hip.state(), ora.state, V)
            assert d is None, f"step {t}: {d}"
            np.testing.assert_array_equal(rh[0], ro[0], err_msg=f"obs at step {t}")
            np.testing.assert_array_equal(rh[1], ro[1], err_msg=f"reward at step {t}")
            np.testing.assert_array_equal(rh[2].astype(bool), ro[2], err_msg=f"terminated at step {t}")
            np.testing.assert_array_equal(rh[3].astype(bool), ro[3], err_msg=f"truncated at step {t}")
            np.testing.assert_array_equal(rh[4], ro[4], err_msg=f"episode return at step {t}")
            np.testing.assert_array_equal(rh[5], ro[5], err_msg=f"episode length at step {t}")
            stats["dones"] += int((ro[2] | ro[3]).sum())
            stats["crashes"] += int(ro[2].sum())
            st = ora.state
            stats["lane_changes"] += int((st[_abi.F_LANE, :, 1:V] != st[_abi.F_TLANE, :, 1:V]).sum())
        return stats
    finally:
        hip.close()


@pytest.mark.parametrize("order", ["sorted", "shuffled"])
def test_step_parity_default_config(order):
    cfg = make_cfg(E=48, order=order)
    stats = run_parity(cfg, steps=60, seed=1)
    # the run must actually exercise lane changes, crashes and autoreset
    assert stats["lane_changes"] > 0 and stats["crashes"] > 0 and stats["dones"] > 0, stats


@pytest.mark.parametrize("kind,d", [(_abi.PE_ROPE, 4), (_abi.PE_ROPE, 2), (_abi.PE_DIST, 4),
                                    (_abi.PE_DIST, 2), (_abi.PE_RANK, 4), (_abi.PE_RANK, 16)])
def test_step_parity_fused_wrappers(kind, d):
    cfg = make_cfg(E=24, order="shuffled", pe=kind, d=d)
    table = pe_table_for(kind, d, cfg.obs_vehicles, seed=3)
    run_parity(cfg, steps=25, table=table, seed=2)


def test_step_parity_30_rows_and_truncation():
    # config 3/5 shape (N = 30) and a short horizon so truncation + autoreset happen
    cfg = make_cfg(E=32, order="shuffled", N=30, max_episode_steps=7)
    stats = run_parity(cfg, steps=20, seed=4)
    assert stats["dones"] >= 32


def test_step_parity_dense_crashes():
    # hard steering: many ego crashes / off-road episodes, pile-ups exercise SAT + impacts
    def wild(rng, E, t):
        return np.tanh(rng.normal(size=(E, 2)) * 2.0).astype(np.float32)

    cfg = make_cfg(E=40, vehicles_density=3)
    stats = run_parity(cfg, steps=30, seed=5, action_fn=wild)
    assert stats["crashes"] > 0


def test_step_parity_small_and_odd_sizes():
    for E, vc, lanes in [(1, 50, 4), (3, 10, 2), (5, 63, 5), (7, 0, 1)]:
        cfg = make_cfg(E=E, vehicles_count=vc, lanes_count=lanes)
        run_parity(cfg, steps=8, seed=E)


def test_imported_state_roundtrip_and_step():
    """Edge states (pending impacts, mid-lane-change, crashed cars) injected into both sides."""
    cfg = make_cfg(E=16)
    ora = OracleEnv(cfg)
    ora.reset()
    rng = np.random.default_rng(7)
    st = ora.state.copy()
    V = cfg.vehicles_count + 1
    # crash some cars, give others pending impacts and target lanes
    fl = st[_abi.F_FLAGS]
    crash = rng.random((16, 64)) < 0.05
    fl[:, :V] |= np.where(crash[:, :V], _abi.FLAG_CRASHED, 0).astype(np.uint32)
    imp = rng.random((16, 64)) < 0.05
    fl[:, :V] |= np.where(imp[:, :V], _abi.FLAG_IMPACT, 0).astype(np.uint32)
    st[_abi.F_IMPX][:, :V] = np.where(imp[:, :V], rng.normal(size=(16, V)).astype(np.float32), 0).view(np.uint32)
    tl = st[_abi.F_TLANE].astype(np.int64)
    lane = st[_abi.F_LANE].astype(np.int64)
    chg = rng.random((16, 64)) < 0.2
    newtl = np.clip(lane + rng.choice([-1, 1], size=lane.shape), 0, 3)
    tl = np.where(chg, newtl, tl)
    st[_abi.F_TLANE][:, 1:V] = tl[:, 1:V].astype(np.uint32)
    ora.state[...] = st
    hip = HipEnv(cfg)
    try:
        hip.set_state(st)
        assert diff_state(hip.state(), st, V) is None
        for t in range(10):
            a = policy_actions(rng, 16, t)
            hip.step(a)
            ora.step(a)
            d = diff_state(hip.state(), ora.state, V)
            assert d is None, f"step {t}: {d}"
    finally:
        hip.close()


def _same_words(a, b, V):
    """diff_state with every NaN word equal to every other (payloads are not specified)."""
    a = a.view(np.uint32).copy()
    b = b.view(np.uint32).copy()
    for x in (a, b):
        f = x[:9].view(np.float32)
        f[np.isnan(f)] = np.float32(np.nan)
    return diff_state(a, b, V)


def test_equal_positions_and_nan():
    """Vehicles sharing an x (the reference's neighbour search breaks such ties by list order:
    front = the last of the nearest-ahead, rear = the first of the nearest-behind), -0/+0,
    groups of three, the ego in a tie, and a NaN position."""
    E = 24
    cfg = make_cfg(E=E)
    ora = OracleEnv(cfg)
    ora.reset()
    rng = np.random.default_rng(11)
    st = ora.state.copy()
    V = cfg.vehicles_count + 1
    x = st[_abi.F_X].view(np.float32)
    y = st[_abi.F_Y].view(np.float32)
    spd = st[_abi.F_SPEED].view(np.float32)
    for e in range(16):
        for _ in range(int(rng.integers(3, 8))):
            i, j = rng.choice(V, size=2, replace=False)
            x[e, j] = x[e, i]
            if rng.random() < 0.2:  # same spot and speed: a pile-up starting inside each other
                y[e, j] = y[e, i]
                spd[e, j] = spd[e, i]
    for e in range(16, 20):
        i, j, k = rng.choice(np.arange(1, V), size=3, replace=False)
        x[e, j] = x[e, k] = x[e, i]
    x[20, 3], x[20, 7], x[20, 9] = 0.0, -0.0, 0.0
    x[21, 5] = x[21, 0]
    x[21, 12] = x[21, 0]
    x[22, 4] = np.nan
    x[23, 17] = np.nan
    x[23, 18] = x[23, 19]
    ora.state[...] = st
    hip = HipEnv(cfg)
    try:
        hip.set_state(st)
        for t in range(12):
            a = policy_actions(rng, E, t)
            hip.step(a)
            ora.step(a)
            d = _same_words(hip.state(), ora.state, V)
            assert d is None, f"step {t}: {d}"
    finally:
        hip.close()


_FULL_SIZE = [(4096, None, "sorted", _abi.PE_NONE, 0),      # configs[1]
              (16384, 30, "shuffled", _abi.PE_ROPE, 4),   # configs[2] (rotate_dim 4: d <= F)
              (8192, None, "sorted", _abi.PE_NONE, 0)]    # configs[3]: one GPU's slice of 65536
# configs[4]: 32768 envs per GPU, 30 observed vehicles, the full PE sweep (d_embed 4 <= F)
_FULL_SIZE += [(32768, 30, order, pe, 0 if pe == _abi.PE_NONE else 4)
               for order in ("sorted", "shuffled")
               for pe in (_abi.PE_NONE, _abi.PE_RANK, _abi.PE_DIST, _abi.PE_ROPE)]


@pytest.mark.parametrize("E,N,order,pe,d", _FULL_SIZE)
def test_full_size_env_blocks_match_oracle(E, N, order, pe, d):
    """BASELINE configs[1] / [2] / [3] (per-GPU slice) / [4] (per-GPU slice, every PE kind and
    order) at full size: the whole batch steps on the GPU with autoreset, and three 16-env
    blocks (start, middle, end) are replayed on the oracle from the GPU's reset state with the
    blocks' global env indices (env_offset) -- every word equal."""
    cfg = make_cfg(E=E, order=order, pe=pe, d=d, N=N)
    table = pe_table_for(pe, d, cfg.obs_vehicles) if pe != _abi.PE_NONE else None
    hip = HipEnv(cfg, table)
    steps = 6
    try:
        hip.reset()
        st0 = hip.state()
        rng = np.random.default_rng(11)
        acts = [rng.uniform(-1, 1, (E, 2)).astype(np.float32) for _ in range(steps)]
        outs = []
        for a in acts:
            o = hip.step(a)
            outs.append(tuple(x.copy() for x in o))
        st_end = hip.state()
    finally:
        hip.close()
    V = cfg.vehicles_count + 1
    B = 16
    for off in (0, E // 2 - B // 2, E - B):
        sub = make_cfg(E=B, order=order, pe=pe, d=d, N=N)
        sub.env_offset = off
        sub.seed_stride = cfg.seed_stride
        ora = OracleEnv(sub, table)
        ora.state[:] = st0[:, off:off + B, :]
        for t, a in enumerate(acts):
            ro = ora.step(a[off:off + B])
            rh = outs[t]
            np.testing.assert_array_equal(rh[0][off:off + B], ro[0], err_msg=f"obs, block {off} step {t}")
            np.testing.assert_array_equal(rh[1][off:off + B], ro[1], err_msg=f"reward, block {off}")
            np.testing.assert_array_equal(rh[2][off:off + B].astype(bool), ro[2])
            np.testing.assert_array_equal(rh[3][off:off + B].astype(bool), ro[3])
        d_ = diff_state(st_end[:, off:off + B, :], ora.state, V)
        assert d_ is None, f"block {off}: {d_}"


@pytest.mark.parametrize("E", [4096, 32768])
def test_hip_reset_layout_known_answer(E):
    """The HIP reset at full size against upstream create_random's numbers (the oracle-side
    KAT is tests/test_oracle_env.py::test_reset_layout_known_answer_create_random): every gap
    within offset * [0.9, 1.1] and the sample spanning that range; speeds 25 / U[21, 24)."""
    cfg = make_cfg(E=E, autoreset=False)
    hip = HipEnv(cfg)
    try:
        hip.reset()
        st = hip.state()
    finally:
        hip.close()
    V = cfg.vehicles_count + 1
    x = st[_abi.F_X, :, :V].view(np.float32).astype(np.float64)
    spd = st[_abi.F_SPEED, :, :V].view(np.float32).astype(np.float64)
    spacing = np.full(V, 0.5)
    spacing[0] = 2.0
    offset = spacing[None, :] * (12.0 + spd) * np.exp(-5.0 / 40.0 * cfg.lanes_count)
    prev = np.concatenate([3.0 * offset[:, :1], np.maximum.accumulate(x, axis=1)[:, :-1]], 1)
    j = (x - prev) / offset
    assert j.min() >= 0.9 - 2e-4 and j.max() <= 1.1 + 2e-4, (j.min(), j.max())
    assert j.min() < 0.901 and j.max() > 1.099
    # U(21, 24) in binary32: 21 + 3 * (1 - 2^-24) rounds to 24.0
    assert np.all(spd[:, 0] == 25.0) and spd[:, 1:].min() >= 21.0 and spd[:, 1:].max() <= 24.0
