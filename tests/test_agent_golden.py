"""This build's ActorCritic / PPOAgent.update against the reference's own outputs
(tests/golden/ppo_agent.npz from ppo/agent.py), torch on the CPU.  GAE comes from the oracle
here (the product GAE is the HIP kernel: tests/test_agent_gpu.py runs it for real)."""

import numpy as np
import pytest
import torch

from agent_util import compare, load, oracle_gae, replay_update


def test_actor_critic_forward_evaluate_match_reference():
    from ppo.agent import ActorCritic

    g, _ = load()
    ac = ActorCritic(60, 2, hidden_dim=64)
    ac.load_state_dict({k[5:]: torch.as_tensor(g[k]) for k in g.files if k.startswith("ac_w_")})
    x, z = torch.as_tensor(g["ac_x"]), torch.as_tensor(g["ac_z"])
    with torch.no_grad():
        mean, std, value = ac(x)
        lp, v2, ent = ac.evaluate(x, torch.tanh(z), z)
    np.testing.assert_allclose(mean.numpy(), g["ac_mean"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(std.numpy(), g["ac_std"], rtol=1e-6)
    np.testing.assert_allclose(value.numpy(), g["ac_value"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(lp.numpy(), g["ac_logp"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(ent.numpy(), g["ac_entropy"], rtol=1e-6)
    a, zz, lpd, vd = ac.get_action(g["ac_x"][0], deterministic=True)
    np.testing.assert_allclose(a, g["ac_det_action"], rtol=1e-6, atol=1e-7)
    assert lpd is None
    np.testing.assert_allclose(vd, g["ac_det_value"], rtol=1e-6, atol=1e-6)


def test_state_dict_keys_are_reference_keys():
    from ppo.agent import ActorCritic

    g, _ = load()
    ref = sorted(k[5:] for k in g.files if k.startswith("ac_w_"))
    assert sorted(ActorCritic(60, 2, 64).state_dict().keys()) == ref


@pytest.mark.parametrize("name", ["upd_a", "upd_b"])
def test_ppo_update_matches_reference(name):
    """Full update: same init weights, memory, permutation -> same final weights and metrics."""
    agent, metrics, g, m = replay_update(name, "cpu", gae_fn=oracle_gae)
    compare(agent, metrics, g, m, name, wtol=2e-5)


@pytest.mark.parametrize("name", ["upd_c1", "upd_c2", "upd_c4"])
def test_ppo_update_matches_reference_at_bench_learners(name):
    """The reference's update at the benched learners (ppo_agent_bench.npz: sd 60 / h256,
    sd 120 / h256, sd 120 / h512; 2,048 samples, 8 epochs x 32 minibatches of 64) replayed by
    this build's torch learner on the CPU: final weights and metrics bit for bit, so the golden
    fixtures the GPU test replays (test_fused_update_replays_reference_golden_bench) pin this
    build's own update semantics exactly."""
    agent, metrics, g, m = replay_update(name, "cpu", gae_fn=oracle_gae, bench=True)
    for k, v in agent.actor_critic.state_dict().items():
        np.testing.assert_array_equal(v.detach().numpy(), g[f"{name}_final_{k}"], err_msg=k)
    for k, want in m["metrics"].items():
        assert metrics[k] == want, (k, metrics[k], want)


def test_checkpoint_roundtrip(tmp_path):
    from ppo.agent import PPOAgent

    a = PPOAgent(60, 2, hidden_dim=32)
    p = str(tmp_path / "ck.pth")
    a.save(p)
    b = PPOAgent(60, 2, hidden_dim=32)
    b.load(p)
    for (k, v), (k2, v2) in zip(a.actor_critic.state_dict().items(), b.actor_critic.state_dict().items()):
        assert k == k2 and torch.equal(v, v2)
