"""HighwayEnv: the one-env, numpy-in/numpy-out facade of HighwayVecEnv.

This is what ``make_env`` returns when no ``num_envs`` override is given, so the reference's
own training loop (training/routine.py:121-151: per-episode ``env.reset(seed=...)``, numpy
``flat_state``, Python-float rewards) runs unchanged on the MI355X env.  Each call still executes
the HIP step kernel (E = 1) and synchronises once to hand numpy arrays back; use HighwayVecEnv
(``env_overrides={"num_envs": E}``) for throughput.
"""

from __future__ import annotations

from typing import Any, Dict, Optional

import numpy as np
import torch

from .gym import Env, spaces
from .vec_env import HighwayVecEnv


class HighwayEnv(Env):
    """gymnasium-style single highway-v0 env backed by libhwy.so."""

    metadata = {"render_modes": []}

    def __init__(self, config: Dict[str, Any], device: Optional[torch.device] = None):
        self._vec = HighwayVecEnv(config, num_envs=1, device=device, autoreset=False)
        self.config = self._vec.config
        self.action_space = spaces.Box(-1.0, 1.0, shape=(2,), dtype=np.float32)
        self.observation_space = self._vec.single_observation_space
        self._episode = 0
        self._seed_base = 0
        self._act = torch.zeros(1, 2, dtype=torch.float32, device=self._vec.device)
        self._seed_t = torch.zeros(1, dtype=torch.int64, device=self._vec.device)

    @property
    def device(self) -> torch.device:
        return self._vec.device

    @property
    def vec_env(self) -> HighwayVecEnv:
        return self._vec

    @property
    def max_episode_steps(self) -> int:
        return self._vec.max_episode_steps

    def enable_pe(self, kind, d, table, ego_idx=0, max_dist=100.0):
        self._vec.enable_pe(kind, d, table, ego_idx=ego_idx, max_dist=max_dist)
        self.observation_space = self._vec.single_observation_space

    def set_pe_table(self, table):
        self._vec.set_pe_table(table)

    def reset(self, *, seed: Optional[int] = None, options: Optional[dict] = None):
        """``seed`` seeds this episode's traffic (gymnasium reset(seed=...) semantics)."""
        if seed is None:
            # gymnasium continues the env's RNG stream; here: next seed of the schedule
            self._episode += 1
            seed = self._seed_base + self._episode
        else:
            self._seed_base, self._episode = int(seed), 0
        self._seed_t.fill_(int(seed))
        obs, _ = self._vec.reset(seeds=self._seed_t)
        return obs[0].cpu().numpy(), {}

    def step(self, action):
        a = torch.as_tensor(np.asarray(action, dtype=np.float32).reshape(1, 2))
        self._act.copy_(a, non_blocking=False)
        obs, rew, term, trunc, _ = self._vec.step(self._act)
        host = torch.cat([rew.view(1), term.view(1).float(), trunc.view(1).float()]).cpu().numpy()
        return (obs[0].cpu().numpy(), float(host[0]), bool(host[1] > 0), bool(host[2] > 0), {})

    def close(self):
        self._vec.close()
