"""make_env -- builds the (wrapped) highway-v0 env for an experiment condition.

Same signature, config resolution and errors as the reference's experiments/wrappers.py:14-104:
  1. deep-copy ``base_cfg`` and deep-merge ``env_overrides`` (:33-44);
  2. resolve the row order with ``setdefault`` per condition (:47-57) -- including the
     reference's quirk that a base config which already says ``"order": "sorted"`` keeps sorted
     rows for the SHUFFLED* conditions; pass
     ``env_overrides={"observation": {"order": "shuffled"}}`` for truly shuffled rows;
  3. reject odd / too-large ``d_embed`` for DistPE and RoPE (:60-71, :85-88);
  4. build the env (gym.make("highway-v0") in the reference, :80 -- the MI355X env here);
  5. wrap with RankEmbedWrapper / DistanceEmbedWrapper / RotaryEmbedWrapper (:91-104).

Extra (native-only) keys read from the merged config, all optional:
  ``num_envs``        lockstep envs on this GPU; > 1 returns a HighwayVecEnv (torch tensors),
                      1 (default) the numpy single-env facade the reference's routine expects
  ``device``          HIP device (default: current)
  ``autoreset``       vector env only, default True
  ``env_offset``, ``global_envs``   episode-seed schedule for env-sharded multi-GPU runs
  ``max_episode_steps``             horizon override (see hwy/_abi.py)
"""

from __future__ import annotations

import copy
from typing import Any, Dict, Optional

from hwy.single_env import HighwayEnv
from hwy.vec_env import HighwayVecEnv

from .config import Condition
from .dist_embed import DistanceEmbedWrapper
from .rank_embed import RankEmbedWrapper
from .rope_embed import RotaryEmbedWrapper

_NATIVE_KEYS = ("num_envs", "device", "autoreset", "env_offset", "global_envs")

_SHUFFLED_FAMILY = (
    Condition.SHUFFLED,
    Condition.SHUFFLED_RANKPE,
    Condition.SHUFFLED_DISTPE,
    Condition.SHUFFLED_ROPE,
)


def _deep_update(orig: Dict[str, Any], updates: Dict[str, Any]) -> None:
    for key, val in updates.items():
        if key in orig and isinstance(orig[key], dict) and isinstance(val, dict):
            _deep_update(orig[key], val)
        else:
            orig[key] = val


def _check_even_le(d_embed: Optional[int], F: int, msg: str) -> None:
    if d_embed is not None and (d_embed % 2 != 0 or d_embed > F):
        raise ValueError(msg)


def resolve_config(exp_condition: Condition, base_cfg: Dict[str, Any],
                   d_embed: Optional[int] = None, env_overrides: Optional[Dict[str, Any]] = None):
    """Steps 1-3 of make_env (no device work): returns (env config, native-only options)."""
    cfg = copy.deepcopy(base_cfg)
    _deep_update(cfg, copy.deepcopy(env_overrides or {}))

    obs_cfg = cfg.setdefault("observation", {})
    if exp_condition is Condition.SORTED:
        obs_cfg.setdefault("order", "sorted")
    elif exp_condition in _SHUFFLED_FAMILY:
        obs_cfg.setdefault("order", "shuffled")

    n_feat = len(cfg["observation"].get("features", []))
    if exp_condition is Condition.SHUFFLED_DISTPE:
        _check_even_le(d_embed, n_feat, "d_embed must be even and ≤ feature count for DistPE")
    if exp_condition is Condition.SHUFFLED_ROPE:
        _check_even_le(d_embed, n_feat, "rotate_dim (d_embed) must be even and ≤ feature count")

    native = {k: cfg.pop(k) for k in _NATIVE_KEYS if k in cfg}
    return cfg, native


def make_env(exp_condition: Condition, base_cfg: Dict[str, Any], d_embed: Optional[int] = None,
             env_overrides: Dict[str, Any] = {}):  # noqa: B006 - reference signature
    cfg, native = resolve_config(exp_condition, base_cfg, d_embed, env_overrides)
    num_envs = int(native.get("num_envs", 1))
    if num_envs > 1:
        env = HighwayVecEnv(cfg, num_envs=num_envs, device=native.get("device"),
                            autoreset=bool(native.get("autoreset", True)),
                            env_offset=int(native.get("env_offset", 0)),
                            global_envs=native.get("global_envs"))
    else:
        env = HighwayEnv(cfg, device=native.get("device"))

    F = env.observation_space.shape[1]
    if exp_condition is Condition.SHUFFLED_ROPE and d_embed is not None:
        if d_embed % 2 or d_embed > F:
            raise ValueError(f"rotate_dim / d_embed must be even and ≤ {F}")

    if exp_condition is Condition.SHUFFLED_RANKPE:
        if d_embed is None:
            raise ValueError("d_embed must be specified for SHUFFLED_RANKPE")
        return RankEmbedWrapper(env, d_embed=d_embed)
    if exp_condition is Condition.SHUFFLED_DISTPE:
        if d_embed is None:
            raise ValueError("d_embed must be specified for SHUFFLED_DISTPE")
        return DistanceEmbedWrapper(env, d_embed=d_embed)
    if exp_condition is Condition.SHUFFLED_ROPE:
        return RotaryEmbedWrapper(env, rotate_dim=d_embed)
    return env
