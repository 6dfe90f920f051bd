"""ExperimentRunner.launch_group's argument checks (experiments/runner.py), without a GPU: the
experiments of one grouped job may differ only in seed and name, and the grouped job needs the
vectorised loop (the reference's one-env loop, launch() with num_envs 1, is not grouped)."""

import pytest


def _exp(seed, **kw):
    from experiments.config import Condition, ConditionHP, Experiment

    hp = ConditionHP(lr=3e-4, clip_eps=0.2, epochs=2, batch_size=64,
                     hidden_dim=kw.pop("hidden_dim", 256), d_embed=None)
    hp.steps_per_update = 16 * 32
    extra = {"num_envs": kw.pop("num_envs", 16), "num_minibatches": 8, "eval_interval": 8}
    return Experiment(name=f"g{seed}", condition=kw.pop("condition", Condition.SORTED), hp=hp,
                      seed=seed, max_episodes=kw.pop("max_episodes", 24), target_reward=1e9,
                      extra=extra, env_config_overrides={})


def test_launch_group_rejects_experiments_that_differ_beyond_seed():
    from config.base_config import HIGHWAY_CONFIG
    from experiments.config import Condition
    from experiments.runner import ExperimentRunner

    r = ExperimentRunner(HIGHWAY_CONFIG)
    with pytest.raises(ValueError, match="differ only in seed"):
        r.launch_group([_exp(42), _exp(1042, hidden_dim=384)])
    with pytest.raises(ValueError, match="differ only in seed"):
        r.launch_group([_exp(42), _exp(1042, condition=Condition.SHUFFLED_ROPE)])
    with pytest.raises(ValueError, match="differ only in seed"):
        r.launch_group([_exp(42), _exp(1042, max_episodes=48)])


def test_launch_group_needs_the_vectorised_loop():
    from config.base_config import HIGHWAY_CONFIG
    from experiments.runner import ExperimentRunner

    with pytest.raises(ValueError, match="num_envs"):
        ExperimentRunner(HIGHWAY_CONFIG).launch_group([_exp(42, num_envs=1),
                                                       _exp(1042, num_envs=1)])
