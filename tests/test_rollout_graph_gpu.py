"""ppo/rollout.py: the lockstep rollout replayed as one HIP graph equals the eager launch
sequence bit for bit, across updates (the acting kernel then streams the update's tile image)
and across a launch-configuration change (seed schedule), which forces a re-capture."""

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _setup(use_graph, E=256, T=8):
    from config.base_config import HIGHWAY_CONFIG
    from hwy.vec_env import HighwayVecEnv
    from ppo.agent import PPOAgent, RolloutBuffer
    from ppo.rollout import LockstepRollout

    torch.manual_seed(3)
    env = HighwayVecEnv(HIGHWAY_CONFIG, num_envs=E, device=DEV, autoreset=True, seed_base=11)
    agent = PPOAgent(60, 2, lr=3e-4, epochs=2, hidden_dim=64, device=DEV, num_minibatches=4,
                     seed=5)
    buf = RolloutBuffer(T, E, 60, 2, DEV)
    obs, _ = env.reset()
    buf.states[0].copy_(obs.reshape(E, 60))
    return env, agent, buf, LockstepRollout(agent, env, buf, use_graph=use_graph)


def test_graph_rollout_equals_eager():
    runs = []
    for use_graph in (False, True):
        env, agent, buf, roll = _setup(use_graph)
        snaps = []
        for it in range(5):
            if it == 3:  # launch configuration change: re-capture
                env.set_seed_schedule(99)
            roll.run()
            snaps.append(torch.cat([buf.states.flatten(), buf.actions.flatten(),
                                    buf.log_probs.flatten(), buf.values.flatten(),
                                    buf.rewards.flatten(), buf.dones.float().flatten(),
                                    buf.ep_return.flatten()]).clone())
            agent.update_rollout(buf, agent.value(buf.states[buf.T]))
            buf.states[0].copy_(buf.states[buf.T])
        torch.cuda.synchronize()
        if use_graph:
            assert roll._graph is not None  # replays happened
        runs.append(snaps)
        env.close()
    for it, (a, b) in enumerate(zip(*runs)):
        assert torch.equal(a, b), it
