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


def test_training_routine_single_env_reference_loop(tmp_path, monkeypatch):
    from config.base_config import HIGHWAY_CONFIG
    from experiments.config import Condition
    from experiments.wrappers import make_env
    from ppo.agent import PPOAgent
    from training.routine import train_with_experiment_name

    monkeypatch.chdir(tmp_path)
    env = make_env(Condition.SORTED, HIGHWAY_CONFIG)
    agent = PPOAgent(60, 2, epochs=1, hidden_dim=32, device=torch.device("cuda", 0), use_graphs=False)
    rewards, avg, mh = train_with_experiment_name(env, agent, max_episodes=4, target_reward=1e9,
                                                  eval_interval=2, steps_per_update=64,
                                                  experiment_name="t_one", exp_seed=42)
    assert len(rewards) == 3 and mh["episode_numbers"][:4] == [1, 2, 3, 4]
    env.close()
