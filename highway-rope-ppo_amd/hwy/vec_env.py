"""HighwayVecEnv: thousands of lockstep highway-v0 envs on one MI355X, behind libhwy.so.

Replaces ``gym.make("highway-v0", config=cfg)`` (experiments/wrappers.py:80) with a batched,
device-resident env.  ``reset`` / ``step`` mirror the gymnasium 1.x contract the reference's
training loop uses (training/routine.py:18-26,127-135) with a leading env axis and torch device
tensors instead of numpy:

    obs, info = env.reset(seed=base)                     # obs: [E, N, F_out] float32
    obs, reward, terminated, truncated, info = env.step(actions)   # actions: [E, 2] in [-1, 1]

With ``autoreset=True`` finished envs restart inside the step kernel with the next seed of the
episode schedule (include/hwy.h) and ``info["episode_return"/"episode_length"]`` report the
finished episode (0 elsewhere).  Every call is asynchronous on the current HIP stream.
"""

from __future__ import annotations

import ctypes
import copy
from typing import Any, Dict, Optional

import numpy as np
import torch

from . import _abi
from ._abi import HWY_MAX_VEHICLES, NFIELDS, PE_NONE, config_from_dict
from .gym import spaces
from .native import (HwyNativeError, HwyStepGroupPlan, HwyStepIO, check, lib, ptr,
                     stream_ptr)


class HighwayVecEnv:
    """E lockstep highway-v0 envs with state resident in HBM (one wavefront per env)."""

    is_vector_env = True

    def __init__(self, config: Dict[str, Any], num_envs: int = 1,
                 device: Optional[torch.device] = None, autoreset: bool = True,
                 seed_base: int = 0, env_offset: int = 0, global_envs: Optional[int] = None,
                 pe_kind: int = PE_NONE, d_embed: int = 0, pe_table: Optional[np.ndarray] = None,
                 ego_idx: int = 0, pe_max_dist: float = 100.0):
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
        device = torch.device(device)
        if device.type != "cuda":
            raise HwyNativeError(
                f"HighwayVecEnv runs on a HIP device only (got {device}); there is no CPU path")
        if device.index is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.config = copy.deepcopy(config)
        self.device = device
        self.num_envs = int(num_envs)
        self._handle = ctypes.c_void_p()
        self._cfg = config_from_dict(self.config, num_envs=num_envs, autoreset=autoreset,
                                     env_offset=env_offset, seed_base=seed_base,
                                     seed_stride=global_envs if global_envs else num_envs,
                                     pe_kind=pe_kind, d_embed=d_embed, ego_idx=ego_idx,
                                     pe_max_dist=pe_max_dist)
        self._pe_table = None if pe_table is None else np.ascontiguousarray(pe_table, np.float32)
        self._create()
        self._alloc_buffers()
        self.action_space = spaces.Box(-1.0, 1.0, shape=(2,), dtype=np.float32)
        self._set_obs_space()

    # ------------------------------------------------------------------ setup
    def _create(self):
        # bumped whenever a launch argument a captured rollout graph bakes in changes (handle,
        # seed schedule, PE table): ppo/rollout.py re-captures then
        self.launch_version = getattr(self, "launch_version", 0) + 1
        with torch.cuda.device(self.device):
            h = ctypes.c_void_p()
            check(lib().hwy_create(ctypes.byref(self._cfg), self.device.index, ctypes.byref(h)),
                  "hwy_create")
            if self._pe_table is not None and self._pe_table.size:
                rc = lib().hwy_set_pe_table(h, self._pe_table.ctypes.data_as(ctypes.c_void_p),
                                            int(self._pe_table.size))
                if rc:
                    lib().hwy_destroy(h)
                    check(rc, "hwy_set_pe_table")
            self._handle = h

    def _alloc_buffers(self):
        E, N, Fo = self.num_envs, self.obs_rows, self.obs_features
        kw = dict(device=self.device)
        self.obs_buf = torch.zeros(E, N, Fo, dtype=torch.float32, **kw)
        self.reward_buf = torch.zeros(E, dtype=torch.float32, **kw)
        self.term_buf = torch.zeros(E, dtype=torch.uint8, **kw)
        self.trunc_buf = torch.zeros(E, dtype=torch.uint8, **kw)
        self.ep_ret_buf = torch.zeros(E, dtype=torch.float32, **kw)
        self.ep_len_buf = torch.zeros(E, dtype=torch.int32, **kw)

    def _set_obs_space(self):
        N, Fo = self.obs_rows, self.obs_features
        self.single_observation_space = spaces.Box(-np.inf, np.inf, shape=(N, Fo), dtype=np.float32)
        self.observation_space = self.single_observation_space

    @property
    def hwy_config(self) -> _abi.HwyConfig:
        return self._cfg

    @property
    def obs_rows(self) -> int:
        return int(self._cfg.obs_vehicles)

    @property
    def obs_features(self) -> int:
        return self._cfg.obs_features()

    @property
    def max_episode_steps(self) -> int:
        return int(self._cfg.max_steps)

    def enable_pe(self, kind: int, d: int, table: Optional[np.ndarray], ego_idx: int = 0,
                  max_dist: float = 100.0) -> None:
        """Fuse an observation wrapper into the step kernel (keeps the current env state)."""
        if self._cfg.pe_kind != PE_NONE:
            raise ValueError("an observation wrapper is already fused into this env")
        state = self.export_state() if self._handle else None
        old = self._handle
        new_cfg = _abi.HwyConfig.from_buffer_copy(self._cfg)
        new_cfg.pe_kind, new_cfg.d_embed = int(kind), int(d)
        new_cfg.ego_idx, new_cfg.pe_max_dist = int(ego_idx), float(max_dist)
        prev_cfg, prev_table = self._cfg, self._pe_table
        self._cfg = new_cfg
        self._pe_table = None if table is None else np.ascontiguousarray(table, np.float32)
        try:
            self._create()
        except Exception:
            self._cfg, self._pe_table, self._handle = prev_cfg, prev_table, old
            raise
        if old:
            lib().hwy_destroy(old)
        if state is not None:
            self.import_state(state)
        self._alloc_buffers()
        self._set_obs_space()

    def set_pe_table(self, table: np.ndarray) -> None:
        """Replace the fused wrapper's table (e.g. RankEmbedWrapper.to(device))."""
        t = np.ascontiguousarray(table, np.float32)
        torch.cuda.synchronize(self.device)
        check(lib().hwy_set_pe_table(self._handle, t.ctypes.data_as(ctypes.c_void_p), int(t.size)),
              "hwy_set_pe_table")
        self._pe_table = t
        self.launch_version += 1

    # ------------------------------------------------------------------ API
    def reset(self, *, seed: Optional[int] = None, options: Optional[dict] = None,
              seeds: Optional[torch.Tensor] = None, mask: Optional[torch.Tensor] = None):
        """Reset all envs (or those where ``mask`` is set).

        ``seed`` (int) sets the schedule's base: env e starts episode 0 with seed
        ``seed + env_offset + e + 1`` (training/routine.py:127 for E = 1 is seed + episode_num).
        ``seeds`` ([E] int64 tensor) gives explicit per-env seeds instead.
        """
        if seed is not None:
            self.set_seed_schedule(int(seed))
        s = None
        if seeds is not None:
            s = torch.as_tensor(seeds, device=self.device).to(torch.int64).contiguous()
        m = None
        if mask is not None:
            m = torch.as_tensor(mask, device=self.device).to(torch.uint8).contiguous()
        check(lib().hwy_reset(self._handle, ptr(s), ptr(m), ptr(self.obs_buf), stream_ptr()),
              "hwy_reset")
        self._keep = (s, m)
        return self.obs_buf, {}

    def step(self, actions: torch.Tensor):
        a = actions
        if not (a.is_cuda and a.dtype == torch.float32 and a.is_contiguous()):
            a = torch.as_tensor(a, device=self.device, dtype=torch.float32).contiguous()
        if a.numel() != 2 * self.num_envs:
            raise ValueError(f"actions must have {self.num_envs}x2 elements, got {tuple(a.shape)}")
        check(lib().hwy_step(self._handle, ptr(a), ptr(self.obs_buf), ptr(self.reward_buf),
                             ptr(self.term_buf), ptr(self.trunc_buf), ptr(self.ep_ret_buf),
                             ptr(self.ep_len_buf), stream_ptr()), "hwy_step")
        self._keep = a
        info = {"episode_return": self.ep_ret_buf, "episode_length": self.ep_len_buf}
        return self.obs_buf, self.reward_buf, self.term_buf, self.trunc_buf, info

    def step_into(self, actions: torch.Tensor, obs: torch.Tensor, reward: torch.Tensor,
                  terminated: torch.Tensor, truncated: torch.Tensor,
                  ep_return: Optional[torch.Tensor] = None,
                  ep_length: Optional[torch.Tensor] = None) -> None:
        """step() writing straight into caller-owned rollout slices (no copies; graph-safe)."""
        check(lib().hwy_step(self._handle, ptr(actions), ptr(obs), ptr(reward), ptr(terminated),
                             ptr(truncated), ptr(ep_return), ptr(ep_length), stream_ptr()),
              "hwy_step")

    def set_seed_schedule(self, seed_base: int, env_offset: Optional[int] = None,
                          seed_stride: Optional[int] = None) -> None:
        """seed(env e, episode k) = seed_base + env_offset + e + 1 + seed_stride * k."""
        c = self._cfg
        c.seed_base = int(seed_base)
        if env_offset is not None:
            c.env_offset = int(env_offset)
        if seed_stride is not None:
            c.seed_stride = int(seed_stride)
        check(lib().hwy_set_seed_schedule(self._handle, c.seed_base, c.env_offset, c.seed_stride),
              "hwy_set_seed_schedule")
        self.launch_version += 1

    def set_seed_groups(self, seed_bases, envs_per_group: int) -> None:
        """Split the E envs into experiment groups of ``envs_per_group`` consecutive envs, group
        g seeded as a solo handle of that many envs with ``set_seed_schedule(seed_bases[g])``
        would be: seed(env l of group g, episode k) = seed_bases[g] + l + 1 + envs_per_group*k
        (hwy_set_seed_groups; experiments/sweep.py).  ``seed_bases=None`` turns grouping off."""
        if seed_bases is None:
            check(lib().hwy_set_seed_groups(self._handle, None, 0, 1), "hwy_set_seed_groups")
            self._groups = None
        else:
            b = np.ascontiguousarray(np.asarray(seed_bases, dtype=np.int64))
            check(lib().hwy_set_seed_groups(self._handle, b.ctypes.data_as(ctypes.c_void_p),
                                            int(b.size), int(envs_per_group)),
                  "hwy_set_seed_groups")
            c = self._cfg
            c.seed_stride = int(envs_per_group)
            check(lib().hwy_set_seed_schedule(self._handle, c.seed_base, c.env_offset,
                                              c.seed_stride), "hwy_set_seed_schedule")
            self._groups = (b.copy(), int(envs_per_group))
        self.launch_version += 1

    def export_state(self) -> torch.Tensor:
        out = torch.empty(NFIELDS, self.num_envs, HWY_MAX_VEHICLES, dtype=torch.int32,
                          device=self.device)
        check(lib().hwy_export_state(self._handle, ptr(out), stream_ptr()), "hwy_export_state")
        return out

    def import_state(self, state: torch.Tensor) -> None:
        if isinstance(state, np.ndarray):
            state = torch.from_numpy(np.ascontiguousarray(state).view(np.int32))
        st = state.to(self.device)
        if st.dtype != torch.int32:
            raise ValueError("state must be int32/uint32 words")
        st = st.contiguous()
        if st.numel() != NFIELDS * self.num_envs * HWY_MAX_VEHICLES:
            raise ValueError("state has the wrong size")
        check(lib().hwy_import_state(self._handle, ptr(st), stream_ptr()), "hwy_import_state")
        self._keep = st

    def close(self) -> None:
        if self._handle:
            lib().hwy_destroy(self._handle)
            self._handle = ctypes.c_void_p()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    @property
    def unwrapped(self):
        return self


class GroupEnvStep:
    """HighwayVecEnv.step_into for several handles in ONE launch (hwy_step_group): the cells of a
    sweep batch (ppo/group.py GroupBatch), whose handles differ in observation width and fused
    wrapper.  Each env computes exactly what its own handle's step computes.  The launch
    parameters live in a device table per (handle configurations, buffers) key, prepared on first
    use -- outside any graph capture, as GroupBatch's eager first rollout at a key does -- so the
    launch itself is graph-capturable."""

    def __init__(self, envs):
        self.envs = [e.unwrapped if hasattr(e, "unwrapped") else e for e in envs]
        self.n = len(self.envs)
        if self.n < 1:
            raise ValueError("GroupEnvStep needs at least one env")
        self._nb = int(lib().hwy_step_group_table_bytes(self.n))
        self._tables: Dict[Any, Any] = {}

    def launch(self, ios) -> None:
        """ios[i] = (actions, obs, reward, terminated, truncated, ep_return, ep_length) of env i,
        as step_into takes them (the last two may be None)."""
        ptrs = tuple(tuple(ptr(x) for x in io) for io in ios)
        key = (tuple((e._handle.value, e.launch_version) for e in self.envs), ptrs)
        hit = self._tables.get(key)
        if hit is None:
            arr = (HwyStepIO * self.n)()
            for i, p in enumerate(ptrs):
                arr[i] = HwyStepIO(*p)
            hs = (ctypes.c_void_p * self.n)(*[e._handle.value for e in self.envs])
            dev = self.envs[0].device
            t = torch.empty(self._nb, dtype=torch.uint8, device=dev)
            plan = HwyStepGroupPlan()
            check(lib().hwy_step_group_prepare(hs, arr, self.n, t.data_ptr(), ctypes.byref(plan),
                                               stream_ptr()), "hwy_step_group_prepare")
            hit = (t, plan)
            self._tables[key] = hit
        check(lib().hwy_step_group(ctypes.byref(hit[1]), hit[0].data_ptr(), stream_ptr()),
              "hwy_step_group")
