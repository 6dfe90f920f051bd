"""Helpers shared by the parity tests: configs, seeded actions, bit-exact state comparison."""

from __future__ import annotations

import copy

import numpy as np

from config.base_config import HIGHWAY_CONFIG
from hwy import _abi

FIELD_NAMES = ["x", "y", "heading", "speed", "target_speed", "delta", "timer", "impact_x",
               "impact_y", "lane", "target_lane", "flags", "env"]


def make_cfg(E=32, order="sorted", pe=_abi.PE_NONE, d=0, N=None, autoreset=True, seed_base=42,
             **overrides):
    cfg = copy.deepcopy(HIGHWAY_CONFIG)
    cfg["observation"]["order"] = order
    if N is not None:
        cfg["observation"]["vehicles_count"] = N
    cfg.update(overrides)
    return _abi.config_from_dict(cfg, num_envs=E, autoreset=autoreset, seed_base=seed_base,
                                 pe_kind=pe, d_embed=d)


def rope_inv_freq(rotate_dim, base=100.0):
    """experiments/rope_embed.py:36-39 (numpy float32, same expression)."""
    pair_count = rotate_dim // 2
    return (1.0 / (base ** (np.arange(pair_count, dtype=np.float32) / pair_count))).astype(np.float32)


def dist_freqs(d, base=100.0):
    """experiments/dist_embed.py:48-52 (torch float32, same expression)."""
    import torch

    return torch.exp(-torch.arange(0, d, 2, dtype=torch.float32) * (np.log(base) / d)).numpy()


def pe_table_for(kind, d, N, seed=0):
    if kind == _abi.PE_ROPE:
        return rope_inv_freq(d)
    if kind == _abi.PE_DIST:
        return dist_freqs(d)
    if kind == _abi.PE_RANK:
        rng = np.random.default_rng(seed)
        return np.tanh(rng.uniform(-0.05, 0.05, size=(N, d))).astype(np.float32)
    return None


def policy_actions(rng, E, t):
    """Bounded random actions that keep episodes alive for a while (mild steering)."""
    a = np.tanh(rng.normal(size=(E, 2)) * np.array([0.6, 0.15])).astype(np.float32)
    return a


def diff_state(a: np.ndarray, b: np.ndarray, V: int):
    """First differing (field, env, vehicle) between two packed states, or None."""
    a = a.view(np.uint32)
    b = b.view(np.uint32)
    if np.array_equal(a, b):
        return None
    idx = np.argwhere(a != b)
    f, e, v = idx[0]
    fa, fb = a[f, e, v], b[f, e, v]
    if f < 9:
        fa, fb = np.uint32(fa).view(np.float32), np.uint32(fb).view(np.float32)
    return (f"{len(idx)} words differ; first field={FIELD_NAMES[f]} env={e} veh={v}: "
            f"hip={fa!r} oracle={fb!r}")
