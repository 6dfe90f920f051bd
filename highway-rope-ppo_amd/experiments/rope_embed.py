"""RotaryEmbedWrapper -- RoPE on the observation rows (reference experiments/rope_embed.py:6-74).

Rotates feature pairs (x, y), (vx, vy), ... of every row by angles 2*pi*dist*inv_freq, where
dist = clip(||row[:2] - ego_row[:2]|| / max_dist, 0, 1); shape unchanged.  The arithmetic runs
in the HIP kernel (hwy_obs_pe / fused hwy_step); inv_freq is built here exactly as the
reference builds it (numpy float32) and handed to the kernel as a table.
"""

from __future__ import annotations

import numpy as np

from hwy import ops
from utils.defaults import max_dist as _max_dist

from ._pe_base import PEWrapperBase


class RotaryEmbedWrapper(PEWrapperBase):
    pe_kind = ops.PE_ROPE

    def __init__(self, env, rotate_dim: int | None = None, max_dist: float = _max_dist(),
                 base: float | None = None, ego_idx: int = 0):
        super().__init__(env)
        N, F = env.observation_space.shape
        self.rotate_dim = rotate_dim or (F - (F % 2))
        if self.rotate_dim % 2 != 0 or self.rotate_dim > F:
            raise ValueError(f"rotate_dim must be even and ≤ {F}; got {self.rotate_dim}")
        self.max_dist = float(max_dist)
        base = base or self.max_dist
        self.ego_idx = ego_idx
        pairs = self.rotate_dim // 2
        # one inverse frequency per rotated pair, float32 as in rope_embed.py:36-39
        self.inv_freq = (1.0 / (base ** (np.arange(pairs, dtype=np.float32) / pairs))).astype(np.float32)
        self.observation_space = env.observation_space
        self._try_fuse(ego_idx, self.max_dist)

    def _pe_params(self):
        return self.pe_kind, self.rotate_dim, self.inv_freq

    def _apply_rope(self, obs, dist_norm):
        """Rotate pairs of ``obs`` [N, F] by 2*pi*dist_norm*inv_freq (rope_embed.py:44-62).

        ``dist_norm`` is used as given (negative / unclipped values allowed: the reference's
        invertibility test rotates back with -dist_norm)."""
        return self._run(obs, dist_override=dist_norm)
