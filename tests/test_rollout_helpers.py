"""RolloutBuffer's per-rollout helpers and the pre-drawn noise on the torch (CPU) path."""

import torch


def test_cpu_noise_value_dones():
    from ppo.agent import PPOAgent, RolloutBuffer

    torch.manual_seed(0)
    ag = PPOAgent(12, 2, hidden_dim=16, device=torch.device("cpu"), use_graphs=False)
    buf = RolloutBuffer(2, 5, 12, 2, torch.device("cpu"))
    buf.draw_noise(torch.Generator().manual_seed(3))
    assert torch.equal(buf.noise, torch.randn(2, 5, 2, generator=torch.Generator().manual_seed(3)))
    s = torch.randn(5, 12)
    with torch.no_grad():
        a, z, lp, v = ag.select_action(s, noise=buf.noise[0])
        mean, std, val = ag.actor_critic.forward(s)
    torch.testing.assert_close(z, mean + std * buf.noise[0])
    torch.testing.assert_close(a, torch.tanh(z))
    torch.testing.assert_close(ag.value(s), val.squeeze(-1))
    buf.terminated[0, 1] = 1
    buf.truncated[1, 3] = 1
    buf.finish_dones()
    assert buf.dones.nonzero().tolist() == [[0, 1], [1, 3]]
