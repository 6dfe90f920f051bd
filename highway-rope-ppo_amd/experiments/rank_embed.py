"""RankEmbedWrapper -- fixed per-row embedding appended to every observation row
(reference experiments/rank_embed.py:9-51).

The table is an nn.Embedding(N, d) re-initialised U(-0.05, 0.05) from the global torch RNG at
construction (same RNG draws as the reference, so seeded runs build the same table) and is never
trained; each row r gets tanh(W[r]) appended.  The tanh table is computed once (and again after
.to()) and the concatenation runs in the HIP kernel.
"""

from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn

from hwy import ops
from hwy.gym import spaces
from utils.defaults import feature_count as _F

from ._pe_base import PEWrapperBase


class RankEmbedWrapper(PEWrapperBase):
    pe_kind = ops.PE_RANK

    def __init__(self, env, d_embed: int = _F()):
        super().__init__(env)
        space = env.observation_space
        if not isinstance(space, spaces.Box):
            raise TypeError("RankEmbedWrapper requires Box observation space.")
        if len(space.shape) != 2:
            raise ValueError("RankEmbedWrapper requires 2D Box observation space (N, F).")
        N, F = space.shape
        self.d_embed = d_embed
        self.table = nn.Embedding(N, d_embed)
        self.table.weight.data.uniform_(-0.05, 0.05)
        low = np.concatenate([space.low, -np.ones((N, d_embed))], axis=1)
        high = np.concatenate([space.high, np.ones((N, d_embed))], axis=1)
        self.observation_space = spaces.Box(low=low, high=high, shape=(N, F + d_embed), dtype=np.float32)
        self.ego_idx, self.max_dist = 0, 1.0
        self._tanh = self._tanh_table()
        self._try_fuse(0, 1.0)

    def _tanh_table(self) -> np.ndarray:
        with torch.no_grad():
            return torch.tanh(self.table.weight).detach().cpu().numpy().astype(np.float32)

    def _pe_params(self):
        return self.pe_kind, self.d_embed, self._tanh

    def to(self, device):
        """Moves the embedding table (experiments/runner.py:80-84); the tanh table is recomputed
        on that device, as the reference recomputes it each observation."""
        self.table.to(device)
        if torch.device(device).type == "cuda":
            self._device = torch.device(device)
        self._tanh = self._tanh_table()
        if self._fused:
            self.env.set_pe_table(self._tanh)
        return self
