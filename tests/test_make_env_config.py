"""make_env's configuration decisions (reference experiments/wrappers.py:14-104) and the
HIGHWAY_CONFIG -> hwy_config translation -- host logic only, no device."""

import copy

import pytest

from config.base_config import HIGHWAY_CONFIG
from experiments.config import Condition, ConditionHP, expand_condition_hps
from experiments.wrappers import resolve_config
from hwy import _abi


@pytest.mark.parametrize("cond", list(Condition))
def test_setdefault_order_quirk(cond):
    # base config says "sorted": every condition keeps sorted rows
    cfg, _ = resolve_config(cond, HIGHWAY_CONFIG, d_embed=4)
    assert cfg["observation"]["order"] == "sorted"


@pytest.mark.parametrize("cond,want", [(Condition.SORTED, "sorted"), (Condition.SHUFFLED, "shuffled"),
                                       (Condition.SHUFFLED_ROPE, "shuffled")])
def test_order_default_when_base_has_none(cond, want):
    base = copy.deepcopy(HIGHWAY_CONFIG)
    del base["observation"]["order"]
    cfg, _ = resolve_config(cond, base, d_embed=4)
    assert cfg["observation"]["order"] == want


def test_override_deep_merge_and_native_keys():
    cfg, native = resolve_config(Condition.SHUFFLED, HIGHWAY_CONFIG, env_overrides={
        "observation": {"order": "shuffled", "vehicles_count": 30}, "num_envs": 64, "lanes_count": 3})
    assert cfg["observation"]["order"] == "shuffled"
    assert cfg["observation"]["vehicles_count"] == 30
    assert cfg["observation"]["features"] == ["x", "y", "vx", "vy"]  # untouched siblings kept
    assert cfg["lanes_count"] == 3 and native == {"num_envs": 64}
    assert "num_envs" not in cfg
    assert HIGHWAY_CONFIG["observation"]["vehicles_count"] == 15  # base not mutated


@pytest.mark.parametrize("cond,d", [(Condition.SHUFFLED_DISTPE, 3), (Condition.SHUFFLED_DISTPE, 8),
                                    (Condition.SHUFFLED_ROPE, 5), (Condition.SHUFFLED_ROPE, 16)])
def test_d_embed_validation(cond, d):
    with pytest.raises(ValueError):
        resolve_config(cond, HIGHWAY_CONFIG, d_embed=d)


def test_rank_accepts_any_d():
    resolve_config(Condition.SHUFFLED_RANKPE, HIGHWAY_CONFIG, d_embed=16)


def test_config_translation():
    c = _abi.config_from_dict(HIGHWAY_CONFIG, num_envs=7)
    assert (c.num_envs, c.lanes_count, c.vehicles_count, c.obs_vehicles, c.n_features) == (7, 4, 50, 15, 4)
    assert [c.feature_ids[i] for i in range(4)] == [1, 2, 3, 4]
    assert list(c.features_range[0]) == [-100.0, 100.0] and list(c.features_range[2]) == [-30.0, 30.0]
    assert c.order == _abi.ORDER_SORTED and c.absolute == 0 and c.normalize == 1 and c.clip == 1
    assert (c.sim_freq, c.policy_freq, c.max_steps) == (15, 1, 200)
    assert c.vehicles_density == 2.0 and c.ego_spacing == 2.0 and c.initial_lane_id == -1
    assert abs(c.right_lane_reward - 0.1) < 1e-7 and c.collision_reward == -1.0
    assert c.obs_features() == 4
    c2 = _abi.config_from_dict(dict(HIGHWAY_CONFIG, max_episode_steps=40))
    assert c2.max_steps == 40


def test_unsupported_settings_raise():
    bad = copy.deepcopy(HIGHWAY_CONFIG)
    bad["observation"]["features"] = ["x", "long_off"]
    with pytest.raises(ValueError):
        _abi.config_from_dict(bad)
    bad = copy.deepcopy(HIGHWAY_CONFIG)
    bad["action"] = {"type": "DiscreteMetaAction"}
    with pytest.raises(ValueError):
        _abi.config_from_dict(bad)


def test_sweep_expansion_like_reference():
    hp = ConditionHP(sweep={"lr": [1e-4, 3e-4], "hidden_dim": [128, 256, 384], "batch_size": [32, 64]})
    out = expand_condition_hps(hp)
    assert len(out) == 12
    assert (out[0].lr, out[0].hidden_dim, out[0].batch_size) == (1e-4, 128, 32)
    assert (out[-1].lr, out[-1].hidden_dim, out[-1].batch_size) == (3e-4, 384, 64)
    assert all(o.sweep == {} for o in out) and out[0].epochs == 6
