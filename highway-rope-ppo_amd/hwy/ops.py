"""torch-facing entry points of libhwy.so that are not tied to an env handle.

Every function here runs the HIP kernel on the tensor's device and stream; CPU tensors are
rejected (HwyNativeError) -- there is no CPU implementation in the product.
"""

from __future__ import annotations

from typing import Optional, Tuple

import torch

from ._abi import PE_APPENDS, PE_DIST, PE_DIST1, PE_NONE, PE_RANK, PE_ROPE
from .native import check, lib, ptr, require_device, stream_ptr

__all__ = ["obs_pe", "gae", "math_selftest", "PE_NONE", "PE_RANK", "PE_DIST", "PE_ROPE", "PE_DIST1"]


def obs_pe(obs: torch.Tensor, kind: int, d: int, ego_idx: int = 0, max_dist: float = 100.0,
           table: Optional[torch.Tensor] = None,
           dist_override: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Observation wrapper on [..., N, F] float32 -> [..., N, F_out] (hwy_obs_pe)."""
    require_device(obs, "obs")
    if obs.dtype != torch.float32:
        obs = obs.float()
    obs = obs.contiguous()
    *lead, N, F = obs.shape
    E = 1
    for s in lead:
        E *= int(s)
    Fo = F + (d if kind in PE_APPENDS else 0)
    out = torch.empty(*lead, N, Fo, device=obs.device, dtype=torch.float32)
    if table is not None:
        require_device(table, "table")
        table = table.float().contiguous()
    if dist_override is not None:
        require_device(dist_override, "dist_override")
        dist_override = dist_override.float().contiguous()
    check(lib().hwy_obs_pe(ptr(obs), ptr(out), E, N, F, int(kind), int(d), int(ego_idx),
                           float(max_dist), ptr(table), ptr(dist_override), stream_ptr()),
          "hwy_obs_pe")
    return out


def gae(rewards: torch.Tensor, dones: torch.Tensor, values: torch.Tensor,
        last_values: torch.Tensor, gamma: float, lam: float,
        out: Optional[Tuple[torch.Tensor, torch.Tensor]] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """GAE over a [T, E] rollout with float64 arithmetic / float32 storage (hwy_gae)."""
    for t, n in ((rewards, "rewards"), (dones, "dones"), (values, "values"), (last_values, "last_values")):
        require_device(t, n)
    T, E = rewards.shape
    if dones.dtype != torch.uint8:
        dones = dones.to(torch.uint8)
    if out is None:
        adv = torch.empty(T, E, device=rewards.device, dtype=torch.float32)
        ret = torch.empty_like(adv)
    else:
        adv, ret = out
    check(lib().hwy_gae(ptr(rewards.float().contiguous()), ptr(dones.contiguous()),
                        ptr(values.float().contiguous()), ptr(last_values.float().contiguous()),
                        float(gamma), float(lam), T, E, ptr(adv), ptr(ret), stream_ptr()),
          "hwy_gae")
    return adv, ret


def math_selftest(op: int, x: torch.Tensor, y: Optional[torch.Tensor] = None) -> torch.Tensor:
    require_device(x, "x")
    out = torch.empty_like(x)
    check(lib().hwy_math_selftest(int(op), ptr(x), ptr(y), ptr(out), x.numel(), stream_ptr()),
          "hwy_math_selftest")
    return out
