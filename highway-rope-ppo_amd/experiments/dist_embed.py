"""DistanceEmbedWrapper -- sinusoidal distance encoding appended to every observation row
(reference experiments/dist_embed.py:8-96).

Appends [sin(2*pi*d*f_k), cos(2*pi*d*f_k)] for k < d_embed/2 with d the clipped normalised
distance of the row to the ego row (Euclidean over the first two features, or |x - x_ego| when
use_euclidean=False).  freqs are built with torch exactly as the reference does and run through
the HIP kernel.
"""

from __future__ import annotations

import numpy as np
import torch

from hwy import ops
from hwy.gym import spaces
from utils.defaults import max_dist as _max_dist

from ._pe_base import PEWrapperBase


class DistanceEmbedWrapper(PEWrapperBase):
    def __init__(self, env, d_embed: int = 8, max_dist: float = _max_dist(),
                 base: float | None = None, use_euclidean: bool = True, ego_idx: int = 0):
        super().__init__(env)
        space = env.observation_space
        if not isinstance(space, spaces.Box):
            raise TypeError("DistanceEmbedWrapper requires Box observation space.")
        if len(space.shape) != 2:
            raise ValueError("DistanceEmbedWrapper requires 2D Box observation space (N, F).")
        N, F = space.shape
        self.d_embed = d_embed
        if self.d_embed % 2 != 0:
            raise ValueError(f"DistanceEmbedWrapper requires even d_embed; got {self.d_embed}")
        self.max_dist = float(max_dist)
        base = base or self.max_dist
        self.use_euclidean = use_euclidean
        self.ego_idx = ego_idx
        need = 2 if use_euclidean else 1
        if F < need:
            raise ValueError(
                f"DistanceEmbedWrapper requires at least {need} feature(s) for distance "
                f"calculation (features available: {F}).")
        # frequencies exactly as dist_embed.py:48-52 (torch float32)
        self.freqs = torch.exp(-torch.arange(0, d_embed, 2, dtype=torch.float32) * (np.log(base) / d_embed))
        self._freqs_np = self.freqs.cpu().numpy()
        low = np.concatenate([space.low, -np.ones((N, d_embed))], axis=1)
        high = np.concatenate([space.high, np.ones((N, d_embed))], axis=1)
        self.observation_space = spaces.Box(low=low, high=high, shape=(N, F + d_embed), dtype=np.float32)
        self._try_fuse(ego_idx, self.max_dist)

    @property
    def pe_kind(self):
        return ops.PE_DIST if self.use_euclidean else ops.PE_DIST1

    def _pe_params(self):
        return self.pe_kind, self.d_embed, self._freqs_np

    def to(self, device):
        """Kept for runner compatibility (experiments/runner.py:80-84)."""
        self.freqs = self.freqs.to(device)
        self._freqs_np = self.freqs.cpu().numpy()
        if torch.device(device).type == "cuda":
            self._device = torch.device(device)
        return self
