"""ctypes mirror of include/hwy.h and the HIGHWAY_CONFIG -> hwy_config translation.

The translation restates how highway-env 1.10.1 reads the reference's config dict
(config/base_config.py:5-39) after ``make_env``'s deep merge (experiments/wrappers.py:33-57):
the ``observation`` block configures KinematicObservation, the top-level keys configure
HighwayEnv / AbstractEnv.  This module holds no device code and is safe to import anywhere.
"""

from __future__ import annotations

import ctypes
import math
from typing import Any, Dict, Optional

HWY_ABI_VERSION = 1
HWY_MAX_VEHICLES = 64
HWY_MAX_FEATURES = 8
HWY_MAX_OBS_ROWS = 64
HWY_MAX_FOUT = 64

FEATURES = {
    "presence": 0,
    "x": 1,
    "y": 2,
    "vx": 3,
    "vy": 4,
    "cos_h": 5,
    "sin_h": 6,
    "heading": 7,
}
ORDER_SORTED, ORDER_SHUFFLED = 0, 1
PE_NONE, PE_RANK, PE_DIST, PE_ROPE, PE_DIST1 = 0, 1, 2, 3, 4
PE_APPENDS = (PE_RANK, PE_DIST, PE_DIST1)  # kinds that append d columns

# enum hwy_field / hwy_env_word
F_X, F_Y, F_HEADING, F_SPEED, F_TSPEED, F_DELTA, F_TIMER, F_IMPX, F_IMPY = range(9)
F_LANE, F_TLANE, F_FLAGS, F_ENV = 9, 10, 11, 12
NFIELDS = 13
E_STEP, E_EPISODE, E_SEED_LO, E_SEED_HI, E_EGO_ACC, E_EGO_STEER, E_RETURN = range(7)
FLAG_CRASHED, FLAG_IMPACT, FLAG_PRESENT = 1, 2, 4
FLAG_ORDER_SHIFT = 8  # bits 8-13: road-order position (include/hwy.h)
FLOAT_FIELDS = (F_X, F_Y, F_HEADING, F_SPEED, F_TSPEED, F_DELTA, F_TIMER, F_IMPX, F_IMPY)

# Episode horizon in policy steps.  highway-env 1.10.1 truncates on env.time >= duration; the
# reference's own artifacts show an untruncated episode is ~200 policy steps (SURVEY.md §6.4:
# 201-frame demo videos, ~170 mean steps/episode, eval returns up to 144 with per-step reward
# <= 1), which a 40-step reading of duration=40 @ 1 Hz cannot produce.  Default: 5 policy steps
# per second of "duration"; override with the "max_episode_steps" config key.
DEFAULT_STEPS_PER_DURATION = 5


class HwyConfig(ctypes.Structure):
    _fields_ = [
        ("num_envs", ctypes.c_int32),
        ("lanes_count", ctypes.c_int32),
        ("vehicles_count", ctypes.c_int32),
        ("obs_vehicles", ctypes.c_int32),
        ("n_features", ctypes.c_int32),
        ("feature_ids", ctypes.c_int32 * HWY_MAX_FEATURES),
        ("has_range", ctypes.c_int32 * HWY_MAX_FEATURES),
        ("features_range", (ctypes.c_float * 2) * HWY_MAX_FEATURES),
        ("order", ctypes.c_int32),
        ("absolute", ctypes.c_int32),
        ("normalize", ctypes.c_int32),
        ("clip", ctypes.c_int32),
        ("see_behind", ctypes.c_int32),
        ("sim_freq", ctypes.c_int32),
        ("policy_freq", ctypes.c_int32),
        ("max_steps", ctypes.c_int32),
        ("initial_lane_id", ctypes.c_int32),
        ("vehicles_density", ctypes.c_float),
        ("ego_spacing", ctypes.c_float),
        ("speed_limit", ctypes.c_float),
        ("collision_reward", ctypes.c_float),
        ("right_lane_reward", ctypes.c_float),
        ("high_speed_reward", ctypes.c_float),
        ("lane_change_reward", ctypes.c_float),
        ("on_road_reward", ctypes.c_float),
        ("reward_speed_range", ctypes.c_float * 2),
        ("normalize_reward", ctypes.c_int32),
        ("offroad_terminal", ctypes.c_int32),
        ("pe_kind", ctypes.c_int32),
        ("d_embed", ctypes.c_int32),
        ("ego_idx", ctypes.c_int32),
        ("pe_max_dist", ctypes.c_float),
        ("autoreset", ctypes.c_int32),
        ("env_offset", ctypes.c_int32),
        ("seed_base", ctypes.c_int64),
        ("seed_stride", ctypes.c_int64),
    ]

    def obs_features(self) -> int:
        extra = self.d_embed if self.pe_kind in PE_APPENDS else 0
        return int(self.n_features + extra)

    def as_dict(self) -> Dict[str, Any]:
        out = {}
        for name, _ in self._fields_:
            v = getattr(self, name)
            if isinstance(v, ctypes.Array):
                v = [list(x) if isinstance(x, ctypes.Array) else x for x in v]
            out[name] = v
        return out


# highway-env 1.10.1 defaults for keys the reference config may omit (HighwayEnv.default_config,
# AbstractEnv.default_config, KinematicObservation.__init__) [upstream, unverified offline].
_ENV_DEFAULTS = {
    "simulation_frequency": 15,
    "policy_frequency": 1,
    "duration": 40,
    "lanes_count": 4,
    "vehicles_count": 50,
    "initial_lane_id": None,
    "ego_spacing": 2,
    "vehicles_density": 1,
    "collision_reward": -1,
    "right_lane_reward": 0.1,
    "high_speed_reward": 0.4,
    "lane_change_reward": 0,
    "reward_speed_range": [20, 30],
    "normalize_reward": True,
    "offroad_terminal": False,
}
_OBS_DEFAULTS = {
    "vehicles_count": 5,
    "features": ["presence", "x", "y", "vx", "vy"],
    "features_range": None,
    "absolute": False,
    "order": "sorted",
    "normalize": True,
    "clip": True,
    "see_behind": False,
}
MAX_SPEED = 40.0
LANE_WIDTH = 4.0


def default_features_range(lanes_count: int) -> Dict[str, list]:
    """KinematicObservation.normalize_obs defaults when features_range is empty."""
    return {
        "x": [-5.0 * MAX_SPEED, 5.0 * MAX_SPEED],
        "y": [-LANE_WIDTH * lanes_count, LANE_WIDTH * lanes_count],
        "vx": [-2 * MAX_SPEED, 2 * MAX_SPEED],
        "vy": [-2 * MAX_SPEED, 2 * MAX_SPEED],
    }


def config_from_dict(
    cfg: Dict[str, Any],
    num_envs: int = 1,
    pe_kind: int = PE_NONE,
    d_embed: int = 0,
    ego_idx: int = 0,
    pe_max_dist: float = 100.0,
    autoreset: bool = False,
    env_offset: int = 0,
    seed_base: int = 0,
    seed_stride: Optional[int] = None,
) -> HwyConfig:
    """Translate a highway-env config dict (after make_env's merge) into hwy_config.

    Raises ValueError for settings the native env does not implement.
    """
    env = dict(_ENV_DEFAULTS)
    env.update({k: v for k, v in cfg.items() if k not in ("observation", "action")})
    obs = dict(_OBS_DEFAULTS)
    obs.update(cfg.get("observation", {}) or {})
    act = cfg.get("action", {"type": "ContinuousAction"}) or {}

    if obs.get("type", "Kinematics") != "Kinematics":
        raise ValueError(f"observation type {obs.get('type')!r} is not supported (Kinematics only)")
    if act.get("type", "ContinuousAction") != "ContinuousAction":
        raise ValueError(f"action type {act.get('type')!r} is not supported (ContinuousAction only)")
    if not (act.get("longitudinal", True) and act.get("lateral", True)):
        raise ValueError("ContinuousAction must control both longitudinal and lateral")

    c = HwyConfig()
    c.num_envs = int(num_envs)
    c.lanes_count = int(env["lanes_count"])
    c.vehicles_count = int(env["vehicles_count"])
    c.obs_vehicles = int(obs["vehicles_count"])
    feats = list(obs["features"])
    if not 1 <= len(feats) <= HWY_MAX_FEATURES:
        raise ValueError(f"between 1 and {HWY_MAX_FEATURES} features are supported, got {len(feats)}")
    c.n_features = len(feats)
    franges = obs.get("features_range") or default_features_range(c.lanes_count)
    for i, f in enumerate(feats):
        if f not in FEATURES:
            raise ValueError(f"unsupported Kinematics feature {f!r}")
        c.feature_ids[i] = FEATURES[f]
        if f in franges:
            c.has_range[i] = 1
            c.features_range[i][0] = float(franges[f][0])
            c.features_range[i][1] = float(franges[f][1])
    order = obs.get("order", "sorted")
    if order not in ("sorted", "shuffled"):
        raise ValueError(f"observation order must be 'sorted' or 'shuffled', got {order!r}")
    c.order = ORDER_SORTED if order == "sorted" else ORDER_SHUFFLED
    c.absolute = int(bool(obs.get("absolute", False)))
    c.normalize = int(bool(obs.get("normalize", True)))
    c.clip = int(bool(obs.get("clip", True)))
    c.see_behind = int(bool(obs.get("see_behind", False)))
    c.sim_freq = int(env["simulation_frequency"])
    c.policy_freq = int(env["policy_frequency"])
    if "max_episode_steps" in cfg:
        c.max_steps = int(cfg["max_episode_steps"])
    else:
        c.max_steps = int(math.ceil(float(env["duration"]) * DEFAULT_STEPS_PER_DURATION))
    lid = env.get("initial_lane_id")
    c.initial_lane_id = -1 if lid is None else int(lid)
    c.vehicles_density = float(env["vehicles_density"])
    c.ego_spacing = float(env["ego_spacing"])
    c.speed_limit = float(cfg.get("speed_limit", 30.0))
    c.collision_reward = float(env["collision_reward"])
    c.right_lane_reward = float(env["right_lane_reward"])
    c.high_speed_reward = float(env["high_speed_reward"])
    c.lane_change_reward = float(env["lane_change_reward"])
    c.on_road_reward = float(env.get("on_road_reward", 0.0))
    c.reward_speed_range[0] = float(env["reward_speed_range"][0])
    c.reward_speed_range[1] = float(env["reward_speed_range"][1])
    c.normalize_reward = int(bool(env["normalize_reward"]))
    c.offroad_terminal = int(bool(env["offroad_terminal"]))
    c.pe_kind = int(pe_kind)
    c.d_embed = int(d_embed)
    c.ego_idx = int(ego_idx)
    c.pe_max_dist = float(pe_max_dist)
    c.autoreset = int(bool(autoreset))
    c.env_offset = int(env_offset)
    c.seed_base = int(seed_base)
    c.seed_stride = int(num_envs if seed_stride is None else seed_stride)
    return c


def schedule_seed(cfg: HwyConfig, env: int, episode: int) -> int:
    """seed(env e, episode k) of include/hwy.h (= exp_seed + episode_num for one env)."""
    return int(cfg.seed_base + cfg.env_offset + env + 1 + cfg.seed_stride * episode)
