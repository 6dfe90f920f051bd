"""Helpers to replay the reference's golden PPO update with this build's PPOAgent."""

import json
import os

import numpy as np
import torch

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(bench: bool = False):
    """(arrays, meta) of the reference's golden updates: ppo_agent.npz (upd_a / upd_b, small) or,
    bench=True, ppo_agent_bench.npz (upd_c1 / upd_c2 / upd_c4: the benched learners at the
    reference's 2,048-sample, 8-epoch, batch-64 update; make_golden.py bench)."""
    if bench:
        return (np.load(os.path.join(GOLD, "ppo_agent_bench.npz")),
                json.load(open(os.path.join(GOLD, "golden_bench_meta.json"))))
    return np.load(os.path.join(GOLD, "ppo_agent.npz")), json.load(open(os.path.join(GOLD, "golden_meta.json")))


def replay_update(name, device, gae_fn=None, use_graphs=False, bench=False):
    """Build PPOAgent with the golden initial weights and memory, run update() with the same
    minibatch permutation (global numpy RNG seeded as the generator did), return (agent, metrics)."""
    from ppo.agent import PPOAgent

    g, meta = load(bench)
    m = meta["agent"][name]
    agent = PPOAgent(m["state_dim"], 2, lr=m["lr"], epochs=m["epochs"], batch_size=m["batch_size"],
                     hidden_dim=m["hidden_dim"], device=torch.device(device), use_graphs=use_graphs)
    sd = {k[len(name) + 6:]: torch.as_tensor(g[k]) for k in g.files if k.startswith(f"{name}_init_")}
    agent.actor_critic.load_state_dict(sd)
    n = m["n"]
    a = {k: g[f"{name}_{k}"] for k in ("states", "actions", "pre_tanh", "rewards", "log_probs",
                                        "dones", "values")}  # each npz member decompressed once
    for t in range(n):
        agent.memory.store(a["states"][t], a["actions"][t], a["pre_tanh"][t],
                           float(a["rewards"][t]), None, float(a["log_probs"][t]),
                           bool(a["dones"][t]), a["values"][t])
    if gae_fn is not None:
        agent.memory.compute_advantages = gae_fn(agent.memory)
    np.random.seed(m["np_seed"])
    metrics = agent.update(last_value=m["last_value"])
    return agent, metrics, g, m


def oracle_gae(memory):
    from oracle import oracle

    def f(gamma, lam, last_value):
        T = len(memory.rewards)
        adv, ret = oracle.gae(np.asarray(memory.rewards, np.float32).reshape(T, 1),
                              np.asarray(memory.dones, np.uint8).reshape(T, 1),
                              np.asarray(memory.values, np.float32).reshape(T, 1),
                              np.array([last_value], np.float32), gamma, lam)
        return adv[:, 0], ret[:, 0]

    return f


def compare(agent, metrics, g, m, name, wtol):
    for k, v in agent.actor_critic.state_dict().items():
        want = g[f"{name}_final_{k}"]
        np.testing.assert_allclose(v.detach().cpu().numpy(), want, atol=wtol, rtol=wtol, err_msg=k)
    for k, want in m["metrics"].items():
        assert abs(metrics[k] - want) <= 1e-4 * max(1.0, abs(want)), (k, metrics[k], want)
