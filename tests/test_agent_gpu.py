"""PPO on the HIP device: the reference's golden update with the real hwy_gae kernel, graph vs
eager equality of the batched update, and short end-to-end training through the routine."""

import numpy as np
import pytest
import torch

from agent_util import compare, replay_update

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["upd_a", "upd_b"])
def test_ppo_update_on_gpu_matches_reference(name):
    agent, metrics, g, m = replay_update(name, "cuda:0", use_graphs=False)
    compare(agent, metrics, g, m, name, wtol=5e-5)


def test_ppo_update_graph_equals_eager():
    a1, m1, g, m = replay_update("upd_a", "cuda:0", use_graphs=False)
    a2, m2, _, _ = replay_update("upd_a", "cuda:0", use_graphs=True)
    for (k, v1), (_, v2) in zip(a1.actor_critic.state_dict().items(), a2.actor_critic.state_dict().items()):
        torch.testing.assert_close(v1, v2, rtol=1e-6, atol=1e-7, msg=k)
    for k in m1:
        assert abs(m1[k] - m2[k]) <= 1e-6 * max(1, abs(m1[k])), k


def _rollout_agent(use_graphs, seed=0):
    from config.base_config import HIGHWAY_CONFIG
    from hwy.vec_env import HighwayVecEnv
    from ppo.agent import PPOAgent, RolloutBuffer

    torch.manual_seed(seed)
    dev = torch.device("cuda", 0)
    E, T = 128, 16
    env = HighwayVecEnv(HIGHWAY_CONFIG, num_envs=E, device=dev, seed_base=3)
    agent = PPOAgent(60, 2, lr=3e-4, epochs=3, hidden_dim=64, device=dev, num_minibatches=8,
                     use_graphs=use_graphs, seed=seed)
    buf = RolloutBuffer(T, E, 60, 2, dev)
    obs, _ = env.reset()
    buf.states[0].copy_(obs.reshape(E, 60))
    for it in range(2):
        for t in range(T):
            a, z, lp, v = agent.select_action(buf.states[t])
            buf.actions[t].copy_(a)
            buf.pre_tanh[t].copy_(z)
            buf.log_probs[t].copy_(lp)
            buf.values[t].copy_(v)
            env.step_into(buf.actions[t], buf.states[t + 1], buf.rewards[t], buf.terminated[t],
                          buf.truncated[t], buf.ep_return[t], buf.ep_length[t])
            torch.bitwise_or(buf.terminated[t], buf.truncated[t], out=buf.dones[t])
        with torch.no_grad():
            _, _, lv = agent.actor_critic(buf.states[T])
        metrics = agent.update_rollout(buf, lv.squeeze(-1))
        buf.states[0].copy_(buf.states[T])
    env.close()
    return agent, metrics


def test_batched_update_graph_equals_eager():
    a1, m1 = _rollout_agent(False)
    a2, m2 = _rollout_agent(True)
    for (k, v1), (_, v2) in zip(a1.actor_critic.state_dict().items(), a2.actor_critic.state_dict().items()):
        torch.testing.assert_close(v1, v2, rtol=1e-5, atol=1e-6, msg=k)
    assert all(np.isfinite(v) for v in m2.values())


def test_training_routine_vectorised(tmp_path, monkeypatch):
    from config.base_config import HIGHWAY_CONFIG
    from experiments.config import Condition
    from experiments.wrappers import make_env
    from ppo.agent import PPOAgent
    from training.routine import train_with_experiment_name

    monkeypatch.chdir(tmp_path)
    env = make_env(Condition.SORTED, HIGHWAY_CONFIG, env_overrides={"num_envs": 64})
    agent = PPOAgent(60, 2, lr=3e-4, epochs=2, hidden_dim=64, device=torch.device("cuda", 0),
                     num_minibatches=4)
    rewards, avg, mh = train_with_experiment_name(env, agent, max_episodes=120, target_reward=1e9,
                                                  eval_interval=50, steps_per_update=64 * 16,
                                                  experiment_name="t_vec", exp_seed=42)
    assert len(rewards) == len(avg) >= 3  # initial + 2 evals
    assert (tmp_path / "artifacts/highway-ppo/summary_t_vec.csv").exists()
    assert (tmp_path / "artifacts/highway-ppo/checkpoints/ppo_highway_best_t_vec.pth").exists()
    assert mh["policy_updates"] and set(mh) >= {"episode_rewards", "eval_rewards", "timestamps"}
    env.close()


def test_configs0_single_env_reference_loop(tmp_path, monkeypatch, caplog):
    """BASELINE configs[0]: the reference's own one-env loop (training/routine.py:121-243) at the
    config-1 hyperparameters (experiments/config.py:33-37 with hidden_dim 64: lr 1e-4, 6 epochs,
    batch_size 64, 2048 steps per update), sorted observation, no PE.  It runs until at least one
    full 2048-sample update has completed; the update's metrics must be finite and logged in the
    reference's update_complete format (ppo/agent.py:289-298)."""
    import logging
    import re

    from config.base_config import HIGHWAY_CONFIG
    from experiments.config import Condition
    from experiments.wrappers import make_env
    from ppo.agent import PPOAgent
    from training.routine import train_with_experiment_name

    monkeypatch.chdir(tmp_path)
    caplog.set_level(logging.INFO)
    env = make_env(Condition.SORTED, HIGHWAY_CONFIG)
    assert env.observation_space.shape == (15, 4)
    torch.manual_seed(42)
    agent = PPOAgent(60, 2, lr=1e-4, epochs=6, batch_size=64, hidden_dim=64,
                     device=torch.device("cuda", 0))
    rewards, avg, mh = train_with_experiment_name(env, agent, max_episodes=150, target_reward=1e9,
                                                  eval_interval=1000, steps_per_update=2048,
                                                  experiment_name="configs0", exp_seed=42)
    env.close()
    ups = mh["policy_updates"]
    assert any(u["steps"] >= 2048 for u in ups), "no 2048-sample update in 150 episodes"
    keys = ["loss", "policy_loss", "value_loss", "entropy", "clip_fraction", "approx_kl",
            "explained_variance"]
    for u in ups:
        for k in keys:
            assert np.isfinite(u[k]), (k, u)
    fmt = re.compile(r"^update_complete loss=-?\d+\.\d{4} policy_loss=-?\d+\.\d{4} "
                     r"value_loss=-?\d+\.\d{4} entropy=-?\d+\.\d{4} clip_frac=-?\d+\.\d{3} "
                     r"kl=-?\d+\.\d{5} explained_var=-?\d+\.\d{3}$")
    lines = [r.getMessage() for r in caplog.records if r.getMessage().startswith("update_complete")]
    assert len(lines) == len(ups) and all(fmt.match(l) for l in lines), lines[:2]
    assert (tmp_path / "artifacts/highway-ppo/summary_configs0.csv").exists()
