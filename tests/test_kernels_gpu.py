"""Device math library, stand-alone PE kernel and GAE kernel vs the CPU oracle (bit-exact), and
the device math library against libm / numpy in float64."""

import math

import numpy as np
import pytest
import torch

from hwy import _abi, ops
from oracle import oracle
from parity_util import pe_table_for

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _inputs(op, rng, n=200000):
    if op in (0, 1, 2, 8, 11, 12, 13, 14):
        x = np.concatenate([rng.uniform(-4, 4, n // 2), rng.uniform(-2000, 2000, n // 2)])
    elif op == 3:
        x = np.concatenate([rng.uniform(-3, 3, n // 2), rng.normal(0, 1e3, n // 2)])
    elif op == 4:
        x = rng.uniform(-1, 1, n)
    elif op == 5:
        x = rng.uniform(-110, 95, n)
    elif op in (6, 9):
        x = np.abs(rng.normal(0, 100, n)) + 1e-30
    elif op == 7:
        x = np.abs(rng.uniform(0, 4000, n))
    elif op == 15:  # the IDM pow: base >= 0 over every binary32 exponent
        x = (rng.uniform(1, 2, n) * np.exp2(rng.integers(-149, 128, n).astype(np.float64)))
    elif op == 16:  # closest lane: the road, its lane-centre ties (4c + 2) and their neighbours,
        # beyond the road, and |y| around the 2^20 switch to the scan
        ties = np.arange(-8, 40, 2, dtype=np.float32)
        near = np.concatenate([np.nextafter(ties, np.float32(np.inf)),
                               np.nextafter(ties, np.float32(-np.inf))])
        big = np.array([2.0 ** 20, -2.0 ** 20, np.nextafter(np.float32(2.0 ** 20), np.float32(0)),
                        1e9, -1e9, 3e7, 123456.7], np.float32)
        x = np.concatenate([rng.uniform(-20, 40, n - 2 * ties.size - big.size), ties, near[:ties.size],
                            near[ties.size:], big])
    else:
        x = rng.normal(0, 100, n)
    y = None
    if op == 7:
        y = rng.uniform(-4.5, 4.5, n)
    if op == 15:
        y = rng.uniform(3.5, 4.5, n)
    if op == 16:
        y = rng.integers(1, 7, x.size).astype(np.float64)
    if op == 10:
        y = rng.normal(0, 10, n)
    # IEEE special values and range edges ride along with every op
    sp = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e-40, -1e-40, 3.4e38, -3.4e38, 2.0 ** 24,
                   1.0, -1.0, 0.5, np.pi / 2, np.pi, 2 * np.pi], np.float32)
    x = np.concatenate([x, sp])
    if y is not None:
        y = np.concatenate([y, np.full(sp.size, {10: 3.0, 15: 4.0, 16: 4.0}.get(op, 2.0))])
    if op == 15:  # the IDM base is >= 0 (or NaN)
        x = np.where(np.signbit(x), -x, x)
    return x.astype(np.float32), None if y is None else y.astype(np.float32)


@pytest.mark.parametrize("op", list(range(17)))
def test_math_library_bit_exact(op):
    rng = np.random.default_rng(op)
    x, y = _inputs(op, rng)
    host = oracle.math_op(op, x, y)
    xt = torch.as_tensor(x, device=DEV)
    yt = None if y is None else torch.as_tensor(y, device=DEV)
    dev = ops.math_selftest(op, xt, yt).cpu().numpy()
    # NaN payloads differ between the host and the device (x86 vs gfx950 default NaN): NaN == NaN
    bad = np.nonzero((host.view(np.uint32) != dev.view(np.uint32)) & ~(np.isnan(host) & np.isnan(dev)))[0]
    assert bad.size == 0, f"op {op}: {bad.size} mismatches, e.g. x={x[bad[0]]!r} host={host[bad[0]]!r} dev={dev[bad[0]]!r}"


@pytest.mark.parametrize("op,fn,lo,hi,tol", [
    (0, math.sin, -20, 20, 2e-7), (1, math.cos, -20, 20, 2e-7), (3, math.atan, -50, 50, 2e-7),
    (4, math.asin, -1, 1, 3e-7), (5, math.exp, -30, 30, 3e-7), (6, math.log, 1e-3, 1e4, 3e-7),
    (2, math.tan, -1.2, 1.2, 6e-7),
])
def test_device_math_accuracy_against_libm(op, fn, lo, hi, tol):
    """The DEVICE math library against libm in float64: the env kernel and
    the oracle share hwy_math.h, so their bit-exact agreement cannot catch a math-library bug;
    this pins what the gfx950 build computes against an independent reference, at the CPU
    accuracy test's bounds (tests/test_oracle_golden.py), on the ranges the step uses."""
    x = np.random.default_rng(100 + op).uniform(lo, hi, 200000).astype(np.float32)
    got = ops.math_selftest(op, torch.as_tensor(x, device=DEV)).cpu().numpy().astype(np.float64)
    want = np.array([fn(float(v)) for v in x])
    err = np.abs(got - want) / np.maximum(np.abs(want), 1e-30)
    absok = np.abs(got - want) <= 1e-7
    assert np.all((err <= tol) | absok), (float(err.max()), x[np.argmax(err)])


def test_device_pow_and_idm_pow_against_numpy():
    """hm_powf (op 7) and the IDM's hm_powf_idm (op 15) on the device against float64 np.power
    over the IDM's bases (max(v, 0) / v0 <= 2.5) and exponents (DELTA in [3.5, 4.5])."""
    rng = np.random.default_rng(77)
    b = rng.uniform(0, 2.5, 100000).astype(np.float32)
    p = rng.uniform(3.5, 4.5, 100000).astype(np.float32)
    want = np.power(b.astype(np.float64), p.astype(np.float64))
    for op in (7, 15):
        got = ops.math_selftest(op, torch.as_tensor(b, device=DEV),
                                torch.as_tensor(p, device=DEV)).cpu().numpy().astype(np.float64)
        rel = np.abs(got - want) / np.maximum(want, 1e-30)
        assert (rel[want > 1e-30] < 1e-5).all(), (op, float(rel.max()))


@pytest.mark.parametrize("kind,d", [(_abi.PE_NONE, 0), (_abi.PE_ROPE, 4), (_abi.PE_ROPE, 2),
                                    (_abi.PE_DIST, 4), (_abi.PE_DIST, 8), (_abi.PE_RANK, 4),
                                    (_abi.PE_RANK, 3)])
@pytest.mark.parametrize("ego_idx", [0, 2])
def test_obs_pe_kernel_matches_oracle(kind, d, ego_idx):
    rng = np.random.default_rng(kind * 10 + d)
    E, N, F = 300, 15, 4
    obs = rng.uniform(-1, 1, size=(E, N, F)).astype(np.float32)
    obs[:, 10:] = 0.0  # zero-padded rows
    table = pe_table_for(kind, d, N, seed=1)
    want = oracle.obs_pe(obs, kind, d, ego_idx, 100.0, table)
    tt = None if table is None else torch.as_tensor(table, device=DEV)
    got = ops.obs_pe(torch.as_tensor(obs, device=DEV), kind, d, ego_idx, 100.0, tt).cpu().numpy()
    np.testing.assert_array_equal(got, want)


def test_obs_pe_dist_override():
    rng = np.random.default_rng(0)
    obs = rng.normal(size=(5, 6, 4)).astype(np.float32)
    dn = rng.uniform(-1, 1, size=(5, 6)).astype(np.float32)
    table = pe_table_for(_abi.PE_ROPE, 4, 6)
    want = oracle.obs_pe(obs, _abi.PE_ROPE, 4, 0, 1.0, table, dist_override=dn)
    got = ops.obs_pe(torch.as_tensor(obs, device=DEV), _abi.PE_ROPE, 4, 0, 1.0,
                     torch.as_tensor(table, device=DEV),
                     dist_override=torch.as_tensor(dn, device=DEV)).cpu().numpy()
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("T,E", [(1, 1), (7, 3), (64, 4096), (200, 33)])
def test_gae_kernel_matches_oracle(T, E):
    rng = np.random.default_rng(T * 1000 + E)
    rew = rng.uniform(0, 1, size=(T, E)).astype(np.float32)
    val = rng.normal(size=(T, E)).astype(np.float32)
    done = (rng.random((T, E)) < 0.05).astype(np.uint8)
    last = rng.normal(size=E).astype(np.float32)
    a_o, r_o = oracle.gae(rew, done, val, last, 0.99, 0.95)
    t = lambda a: torch.as_tensor(a, device=DEV)  # noqa: E731
    a_h, r_h = ops.gae(t(rew), t(done), t(val), t(last), 0.99, 0.95)
    np.testing.assert_array_equal(a_h.cpu().numpy(), a_o)
    np.testing.assert_array_equal(r_h.cpu().numpy(), r_o)


def test_cpu_tensor_rejected():
    from hwy.native import HwyNativeError

    with pytest.raises(HwyNativeError):
        ops.obs_pe(torch.zeros(1, 3, 4), _abi.PE_ROPE, 4, 0, 100.0, None)
