"""Generate the golden fixtures under tests/golden/ from the reference itself.

Runs ONLY in the build container (needs /root/reference, which never travels to the GPU box):

    python tests/golden/make_golden.py

What is imported from the reference, unmodified:
  * ppo/agent.py (ActorCritic, PPOMemory, PPOAgent) -- imports natively (numpy + torch).
  * experiments/rope_embed.py, dist_embed.py, rank_embed.py and utils/defaults.py -- these
    subclass gymnasium.ObservationWrapper; gymnasium is not installed in this image, so a
    throwaway stand-in providing only the base classes (Env, Wrapper, ObservationWrapper,
    spaces.Box) is written to a temp dir for the duration of this script.  It contributes no
    arithmetic: every number in the fixtures comes from the reference's own methods.
The fixtures are inputs + expected outputs only (npz), no reference source is copied.
"""

from __future__ import annotations

import json
import os
import sys
import tempfile
import textwrap

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))

_SHIM = textwrap.dedent(
    '''
    import numpy as np
    class _Box:
        def __init__(self, low, high, shape=None, dtype=np.float32):
            if shape is None:
                shape = np.broadcast(np.asarray(low), np.asarray(high)).shape
            self.shape = tuple(shape); self.dtype = np.dtype(dtype)
            self.low = np.broadcast_to(np.asarray(low, dtype=self.dtype), self.shape)
            self.high = np.broadcast_to(np.asarray(high, dtype=self.dtype), self.shape)
    class spaces:
        Box = _Box
    class Env:
        observation_space = None
        action_space = None
    class Wrapper(Env):
        def __init__(self, env):
            self.env = env
            self.observation_space = env.observation_space
            self.action_space = env.action_space
    class ObservationWrapper(Wrapper):
        pass
    '''
)


class _DummyEnv:
    def __init__(self, shape):
        import gymnasium

        self.observation_space = gymnasium.spaces.Box(-np.inf, np.inf, shape=shape, dtype=np.float32)
        self.action_space = gymnasium.spaces.Box(-1.0, 1.0, shape=(2,), dtype=np.float32)


def _obs_batch(rng, E, N, F, pad_from):
    """Kinematics-like normalised observations: ego row absolute (x clipped to 1), others
    relative, zero-padded tail rows (the quirk of SURVEY.md §8 a5.q)."""
    obs = rng.uniform(-0.3, 0.3, size=(E, N, F)).astype(np.float32)
    obs[:, 0, 0] = 1.0
    obs[:, 0, 1] = rng.choice([0.0, 0.04, 0.08, 0.12], size=E).astype(np.float32)
    for e in range(E):
        obs[e, pad_from[e]:] = 0.0
    return obs


def gen_pe(rng):
    from experiments.dist_embed import DistanceEmbedWrapper
    from experiments.rank_embed import RankEmbedWrapper
    from experiments.rope_embed import RotaryEmbedWrapper
    import torch

    out = {}
    errors = {}
    for N, F in [(15, 4), (30, 4), (6, 6)]:
        E = 12
        pad = rng.integers(1, N + 1, size=E)
        obs = _obs_batch(rng, E, N, F, pad)
        out[f"obs_{N}x{F}"] = obs
        for rd in [None, 2, 4] + ([6] if F >= 6 else []):
            w = RotaryEmbedWrapper(_DummyEnv((N, F)), rotate_dim=rd)
            y = np.stack([w.observation(o) for o in obs])
            key = f"rope_{N}x{F}_rd{w.rotate_dim}"
            out[key] = y
            out[key + "_inv_freq"] = w.inv_freq.astype(np.float32)
            dn = rng.uniform(-1, 1, size=(E, N)).astype(np.float32)
            out[key + "_dn"] = dn
            out[key + "_applied"] = np.stack([w._apply_rope(o.copy(), d) for o, d in zip(obs, dn)])
        for d in [2, 4, 8]:
            w = DistanceEmbedWrapper(_DummyEnv((N, F)), d_embed=d)
            out[f"dist_{N}x{F}_d{d}"] = np.stack([w.observation(o) for o in obs])
            out[f"dist_{N}x{F}_d{d}_freqs"] = w._freqs_np.astype(np.float32)
        for d in [3, 4, 16]:
            torch.manual_seed(1000 + d)
            w = RankEmbedWrapper(_DummyEnv((N, F)), d_embed=d)
            # RankEmbedWrapper.observation calls .numpy() on a grad-requiring tensor
            # (rank_embed.py:48) and raises RuntimeError as written; under no_grad it runs.
            try:
                w.observation(obs[0])
                errors[f"rank_observation_plain"] = "ok"
            except RuntimeError:
                errors[f"rank_observation_plain"] = "RuntimeError"
            with torch.no_grad():
                out[f"rank_{N}x{F}_d{d}"] = np.stack([w.observation(o) for o in obs])
            out[f"rank_{N}x{F}_d{d}_table"] = torch.tanh(w.table.weight).detach().numpy()
            out[f"rank_{N}x{F}_d{d}_weight"] = w.table.weight.detach().numpy()
    # validation behaviour (ValueError / TypeError at construction)
    for rd in [3, 6, 5]:
        try:
            RotaryEmbedWrapper(_DummyEnv((5, 4)), rotate_dim=rd)
            errors[f"rope_rd{rd}"] = "ok"
        except ValueError:
            errors[f"rope_rd{rd}"] = "ValueError"
    for d in [3, 1]:
        try:
            DistanceEmbedWrapper(_DummyEnv((5, 4)), d_embed=d)
            errors[f"dist_d{d}"] = "ok"
        except ValueError:
            errors[f"dist_d{d}"] = "ValueError"
    return out, errors


def gen_gae(rng):
    from ppo.agent import PPOMemory

    out = {}
    cases = [(1, 0.0), (17, 0.5), (256, -1.25), (2048, 3.0)]
    for i, (T, last) in enumerate(cases):
        m = PPOMemory()
        rew = rng.uniform(0, 1, size=T).astype(np.float32)
        val = rng.normal(size=T).astype(np.float32)
        done = rng.random(T) < (0.1 if T > 1 else 1.0)
        if T > 4:
            done[-1] = bool(i % 2)
        for t in range(T):
            # rewards stored as Python floats (float64) like training/routine.py:134-147
            m.store(None, None, None, float(rew[t]), None, None, bool(done[t]), val[t])
        adv, ret = m.compute_advantages(0.99, 0.95, float(np.float32(last)))
        out[f"gae{i}_rewards"] = rew
        out[f"gae{i}_values"] = val
        out[f"gae{i}_dones"] = done.astype(np.uint8)
        out[f"gae{i}_last"] = np.array([last], np.float32)
        out[f"gae{i}_adv"] = adv.astype(np.float32)
        out[f"gae{i}_ret"] = ret.astype(np.float32)
    return out


def gen_agent(rng):
    import torch

    from ppo.agent import ActorCritic, PPOAgent

    out = {}
    meta = {}
    # ActorCritic forward / evaluate / deterministic get_action
    torch.manual_seed(7)
    ac = ActorCritic(60, 2, hidden_dim=64)
    with torch.no_grad():
        ac.log_std.copy_(torch.tensor([-0.3, 0.2]))
    x = rng.normal(size=(33, 60)).astype(np.float32)
    z = rng.normal(size=(33, 2)).astype(np.float32)
    with torch.no_grad():
        mean, std, value = ac.forward(torch.from_numpy(x))
        lp, v2, ent = ac.evaluate(torch.from_numpy(x), torch.tanh(torch.from_numpy(z)), torch.from_numpy(z))
    for k, v in ac.state_dict().items():
        out[f"ac_w_{k}"] = v.numpy().copy()
    out["ac_x"] = x
    out["ac_z"] = z
    out["ac_mean"] = mean.numpy()
    out["ac_std"] = std.numpy()
    out["ac_value"] = value.numpy()
    out["ac_logp"] = lp.numpy()
    out["ac_entropy"] = ent.numpy()
    a_det, z_det, lp_det, v_det = ac.get_action(x[0], deterministic=True)
    out["ac_det_action"] = np.asarray(a_det, np.float32)
    out["ac_det_value"] = np.asarray(v_det, np.float32)

    # One full PPOAgent.update (ppo/agent.py:196-308)
    for name, (sd, h, epochs, bs, n) in {"upd_a": (60, 64, 2, 64, 256), "upd_b": (60, 32, 3, 50, 130)}.items():
        torch.manual_seed(11)
        agent = PPOAgent(sd, 2, lr=3e-4, epochs=epochs, batch_size=bs, hidden_dim=h)
        init = {k: v.detach().clone().numpy() for k, v in agent.actor_critic.state_dict().items()}
        S = rng.normal(size=(n, sd)).astype(np.float32)
        Zs = rng.normal(size=(n, 2)).astype(np.float32) * 0.7
        with torch.no_grad():
            m_, s_, v_ = agent.actor_critic.forward(torch.from_numpy(S))
            dist = torch.distributions.Normal(m_, s_)
            zt = torch.from_numpy(Zs)
            at = torch.tanh(zt)
            lp_ = (dist.log_prob(zt) - torch.log1p(-at.pow(2) + 1e-6)).sum(-1)
        R = rng.uniform(0, 1, size=n).astype(np.float32)
        D = rng.random(n) < 0.03
        for t in range(n):
            agent.memory.store(S[t], at[t].numpy(), Zs[t], float(R[t]), None,
                               float(lp_[t].item()), bool(D[t]), v_[t].numpy()[0])
        np.random.seed(123)
        perm_rng = np.random.get_state()
        metrics = agent.update(last_value=0.25)
        np.random.set_state(perm_rng)
        idx = np.arange(n, dtype=np.int64)
        np.random.shuffle(idx)
        out[f"{name}_perm"] = idx
        for k, v in init.items():
            out[f"{name}_init_{k}"] = v
        for k, v in agent.actor_critic.state_dict().items():
            out[f"{name}_final_{k}"] = v.detach().numpy()
        out[f"{name}_states"] = S
        out[f"{name}_pre_tanh"] = Zs
        out[f"{name}_actions"] = at.numpy()
        out[f"{name}_log_probs"] = lp_.numpy().astype(np.float32)
        out[f"{name}_rewards"] = R
        out[f"{name}_dones"] = D.astype(np.uint8)
        out[f"{name}_values"] = v_[:, 0].numpy()
        meta[name] = dict(state_dim=sd, hidden_dim=h, epochs=epochs, batch_size=bs, n=n, lr=3e-4,
                          last_value=0.25, np_seed=123, metrics=metrics)
    return out, meta


BENCH_UPDATES = {
    # name: (state_dim, hidden_dim, epochs, batch_size, n) -- the reference's update at the
    # benched learners: configs[1]'s cell (sd 60 / h256), configs[2]'s
    # (sd 120 / h256) and configs[4]'s widest (sd 120 / h512), each at the reference's own
    # update statistics: 2,048 samples, 8 epochs of 32 minibatches of 64 (256 Adam steps)
    "upd_c1": (60, 256, 8, 64, 2048),
    "upd_c2": (120, 256, 8, 64, 2048),
    "upd_c4": (120, 512, 8, 64, 2048),
}


def gen_bench_updates():
    """One full reference PPOAgent.update (ppo/agent.py:196-308) per BENCH_UPDATES entry, with
    its own generator (seed 20261018) so the older fixtures' draws are untouched.  Stored: the
    initial weights, the memory (states, pre-tanh, actions, log-probs, rewards, dones, values),
    the minibatch permutation, the final weights and the metrics dict."""
    import torch

    from ppo.agent import PPOAgent

    rng = np.random.default_rng(20261018)
    out, meta = {}, {}
    for name, (sd, h, epochs, bs, n) in BENCH_UPDATES.items():
        torch.manual_seed(29)
        agent = PPOAgent(sd, 2, lr=3e-4, epochs=epochs, batch_size=bs, hidden_dim=h)
        init = {k: v.detach().clone().numpy() for k, v in agent.actor_critic.state_dict().items()}
        # Kinematics-like inputs: normalised features in [-1, 1], a share of zero-padded rows
        S = np.clip(rng.normal(scale=0.4, size=(n, sd)), -1, 1).astype(np.float32)
        S[rng.random((n, sd)) < 0.15] = 0.0
        Zs = rng.normal(size=(n, 2)).astype(np.float32) * 0.7
        with torch.no_grad():
            m_, s_, v_ = agent.actor_critic.forward(torch.from_numpy(S))
            dist = torch.distributions.Normal(m_, s_)
            zt = torch.from_numpy(Zs)
            at = torch.tanh(zt)
            lp_ = (dist.log_prob(zt) - torch.log1p(-at.pow(2) + 1e-6)).sum(-1)
        R = rng.uniform(0, 1, size=n).astype(np.float32)
        D = rng.random(n) < 0.01
        for t in range(n):
            agent.memory.store(S[t], at[t].numpy(), Zs[t], float(R[t]), None,
                               float(lp_[t].item()), bool(D[t]), v_[t].numpy()[0])
        np.random.seed(321)
        perm_rng = np.random.get_state()
        metrics = agent.update(last_value=0.5)
        np.random.set_state(perm_rng)
        idx = np.arange(n, dtype=np.int64)
        np.random.shuffle(idx)
        out[f"{name}_perm"] = idx
        for k, v in init.items():
            out[f"{name}_init_{k}"] = v
        for k, v in agent.actor_critic.state_dict().items():
            out[f"{name}_final_{k}"] = v.detach().numpy()
        out[f"{name}_states"] = S
        out[f"{name}_pre_tanh"] = Zs
        out[f"{name}_actions"] = at.numpy()
        out[f"{name}_log_probs"] = lp_.numpy().astype(np.float32)
        out[f"{name}_rewards"] = R
        out[f"{name}_dones"] = D.astype(np.uint8)
        out[f"{name}_values"] = v_[:, 0].numpy()
        meta[name] = dict(state_dim=sd, hidden_dim=h, epochs=epochs, batch_size=bs, n=n, lr=3e-4,
                          last_value=0.5, np_seed=321, metrics=metrics)
        print(name, metrics, flush=True)
    return out, meta


def _shim_path():
    tmp = tempfile.mkdtemp(prefix="gym_shim_")
    os.makedirs(os.path.join(tmp, "gymnasium"))
    with open(os.path.join(tmp, "gymnasium", "__init__.py"), "w") as f:
        f.write(_SHIM)
    sys.path[:0] = [REF, tmp]


def main_bench():
    """python tests/golden/make_golden.py bench -> ppo_agent_bench.npz + golden_bench_meta.json"""
    _shim_path()
    import torch

    torch.set_num_threads(1)
    out, meta = gen_bench_updates()
    np.savez_compressed(os.path.join(OUT, "ppo_agent_bench.npz"), **out)
    with open(os.path.join(OUT, "golden_bench_meta.json"), "w") as f:
        json.dump({"agent": meta, "generator": "tests/golden/make_golden.py bench",
                   "reference": "DhruvDh/highway-rope-ppo @ 2025-05-23",
                   "torch": torch.__version__, "numpy": np.__version__,
                   "torch_threads": 1}, f, indent=2)


def main():
    _shim_path()
    import torch

    torch.set_num_threads(1)
    rng = np.random.default_rng(20250523)
    pe, errors = gen_pe(rng)
    np.savez_compressed(os.path.join(OUT, "pe_wrappers.npz"), **pe)
    gae = gen_gae(rng)
    np.savez_compressed(os.path.join(OUT, "gae.npz"), **gae)
    agent, meta = gen_agent(rng)
    np.savez_compressed(os.path.join(OUT, "ppo_agent.npz"), **agent)
    with open(os.path.join(OUT, "golden_meta.json"), "w") as f:
        json.dump({"pe_validation": errors, "agent": meta,
                   "generator": "tests/golden/make_golden.py",
                   "reference": "DhruvDh/highway-rope-ppo @ 2025-05-23",
                   "torch": torch.__version__, "numpy": np.__version__}, f, indent=2)
    print("wrote", sorted(os.listdir(OUT)))


if __name__ == "__main__":
    if sys.argv[1:] == ["bench"]:
        main_bench()
    else:
        main()
