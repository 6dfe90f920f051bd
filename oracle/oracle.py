"""oracle.py -- numpy/ctypes front end of the CPU oracle.  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module:
it is the checker the HIP path is compared against and the timed CPU baseline, never part of
the product path.  The restated algorithms live in hwy_oracle.c (env step/reset/observation,
observation wrappers, GAE) and cite the reference file:line they follow.

Pinning (see DESIGN.md "Oracle"):
  * GAE (ppo/agent.py:126-138) and the PE wrappers (experiments/{rope,dist,rank}_embed.py):
    pinned by tests/golden fixtures generated from the reference itself and by the reference's
    own RoPE tests (tests/test_rope_wrapper.py:34-113) restated as known-answer tests.
  * highway-env 1.10.1 dynamics: third-party, absent offline -> PARITY UNPINNED against
    upstream; pinned only by hand-built known-answer cases (IDM closed form, SAT, sort order).
"""

from __future__ import annotations

import ctypes
import os
import subprocess
import sys
from typing import Optional

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_PKG = os.path.join(os.path.dirname(_HERE), "highway-rope-ppo_amd")
if _PKG not in sys.path:
    sys.path.insert(0, _PKG)

from hwy._abi import (  # noqa: E402
    NFIELDS,
    HWY_MAX_VEHICLES,
    HwyConfig,
)

_LIB_PATH = os.path.join(_HERE, "liboracle_hwy.so")
_lib = None

_f32p = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
_u32p = np.ctypeslib.ndpointer(dtype=np.uint32, flags="C_CONTIGUOUS")
_u8p = np.ctypeslib.ndpointer(dtype=np.uint8, flags="C_CONTIGUOUS")
_u64p = np.ctypeslib.ndpointer(dtype=np.uint64, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")


def build() -> str:
    """Compile liboracle_hwy.so with gcc (oracle/Makefile)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        cfgp = ctypes.POINTER(HwyConfig)
        vp = ctypes.c_void_p
        L.hwyo_reset.argtypes = [cfgp, _u32p, vp, vp, vp, vp]
        L.hwyo_step.argtypes = [cfgp, _u32p, _f32p, _f32p, _f32p, _u8p, _u8p, vp, vp, vp]
        L.hwyo_observe.argtypes = [cfgp, _u32p, _f32p, vp]
        L.hwyo_obs_pe.argtypes = [_f32p, _f32p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                  ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float, vp, vp]
        L.hwyo_gae.argtypes = [_f32p, _u8p, _f32p, _f32p, ctypes.c_double, ctypes.c_double,
                               ctypes.c_int, ctypes.c_int, _f32p, _f32p]
        L.hwyo_math.argtypes = [ctypes.c_int, _f32p, vp, _f32p, ctypes.c_int]
        L.hwyo_philox.argtypes = [_u32p, _u32p, _u32p]
        L.hwyo_philox.restype = None
        L.hwyo_sat_compare.argtypes = [_f32p, ctypes.c_int, _f32p]
        L.hwyo_kin_compare.argtypes = [_f32p, ctypes.c_int, _f32p]
        _lib = L
    return _lib


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


class OracleEnv:
    """Scalar CPU restatement of the vectorised env (same state layout as libhwy.so)."""

    def __init__(self, cfg: HwyConfig, pe_table: Optional[np.ndarray] = None):
        self.cfg = cfg
        self.E = int(cfg.num_envs)
        self.N = int(cfg.obs_vehicles)
        self.Fo = cfg.obs_features()
        self.state = np.zeros((NFIELDS, self.E, HWY_MAX_VEHICLES), dtype=np.uint32)
        self.pe_table = None if pe_table is None else np.ascontiguousarray(pe_table, np.float32)

    def reset(self, seeds: Optional[np.ndarray] = None, mask: Optional[np.ndarray] = None):
        obs = np.zeros((self.E, self.N, self.Fo), dtype=np.float32)
        s = None if seeds is None else np.ascontiguousarray(seeds, np.uint64)
        m = None if mask is None else np.ascontiguousarray(mask, np.uint8)
        lib().hwyo_reset(ctypes.byref(self.cfg), self.state, _ptr(s), _ptr(m), _ptr(obs),
                         _ptr(self.pe_table))
        return obs

    def step(self, actions: np.ndarray):
        a = np.ascontiguousarray(actions, np.float32).reshape(self.E, 2)
        obs = np.zeros((self.E, self.N, self.Fo), dtype=np.float32)
        rew = np.zeros(self.E, np.float32)
        term = np.zeros(self.E, np.uint8)
        trunc = np.zeros(self.E, np.uint8)
        ep_ret = np.zeros(self.E, np.float32)
        ep_len = np.zeros(self.E, np.int32)
        lib().hwyo_step(ctypes.byref(self.cfg), self.state, a, obs, rew, term, trunc,
                        _ptr(ep_ret), _ptr(ep_len), _ptr(self.pe_table))
        return obs, rew, term.astype(bool), trunc.astype(bool), ep_ret, ep_len

    def observe(self):
        obs = np.zeros((self.E, self.N, self.Fo), dtype=np.float32)
        lib().hwyo_observe(ctypes.byref(self.cfg), self.state, obs, _ptr(self.pe_table))
        return obs

    # convenience views
    def field(self, f: int) -> np.ndarray:
        return self.state[f]

    def ffield(self, f: int) -> np.ndarray:
        return self.state[f].view(np.float32)


def obs_pe(obs: np.ndarray, kind: int, d: int, ego_idx: int, max_dist: float,
           table: Optional[np.ndarray], dist_override: Optional[np.ndarray] = None) -> np.ndarray:
    obs = np.ascontiguousarray(obs, np.float32)
    squeeze = obs.ndim == 2
    if squeeze:
        obs = obs[None]
    E, N, F = obs.shape
    Fo = F + (d if kind in (1, 2, 4) else 0)
    out = np.zeros((E, N, Fo), np.float32)
    t = None if table is None else np.ascontiguousarray(table, np.float32)
    dov = None if dist_override is None else np.ascontiguousarray(dist_override, np.float32).reshape(E, N)
    lib().hwyo_obs_pe(obs, out, E, N, F, kind, d, ego_idx, float(max_dist), _ptr(t), _ptr(dov))
    return out[0] if squeeze else out


def gae(rewards, dones, values, last_values, gamma, lam):
    rewards = np.ascontiguousarray(rewards, np.float32)
    T, E = rewards.shape
    adv = np.zeros((T, E), np.float32)
    ret = np.zeros((T, E), np.float32)
    lib().hwyo_gae(rewards, np.ascontiguousarray(dones, np.uint8),
                   np.ascontiguousarray(values, np.float32),
                   np.ascontiguousarray(last_values, np.float32), float(gamma), float(lam), T, E,
                   adv, ret)
    return adv, ret


def math_op(op: int, x: np.ndarray, y: Optional[np.ndarray] = None) -> np.ndarray:
    x = np.ascontiguousarray(x, np.float32)
    out = np.zeros_like(x)
    yy = None if y is None else np.ascontiguousarray(y, np.float32)
    rc = lib().hwyo_math(op, x, _ptr(yy), out, x.size)
    assert rc == 0
    return out


def sat_compare(pairs: np.ndarray) -> np.ndarray:
    """[n, 12] pairs (xa ya ha spa xb yb hb spb dt . . .) -> [n, 8]: upstream's polygon SAT
    (inter, will, tx, ty) and the closed-form rectangle SAT the simulation uses."""
    p = np.ascontiguousarray(pairs, np.float32)
    out = np.zeros((p.shape[0], 8), np.float32)
    assert lib().hwyo_sat_compare(p, p.shape[0], out) == 0
    return out


def kin_compare(rows: np.ndarray) -> np.ndarray:
    """[n, 5] (y, heading, speed, target lane, ego steering) -> [n, 14]: upstream tan of the
    clipped steering, the closed-form steering_tan; (vx, vy, heading rate) upstream / closed
    form for the ego angle, then for the traffic steering."""
    p = np.ascontiguousarray(rows, np.float32)
    out = np.zeros((p.shape[0], 14), np.float32)
    assert lib().hwyo_kin_compare(p, p.shape[0], out) == 0
    return out


def philox(ctr, key) -> np.ndarray:
    out = np.zeros(4, np.uint32)
    lib().hwyo_philox(np.asarray(ctr, np.uint32), np.asarray(key, np.uint32), out)
    return out
