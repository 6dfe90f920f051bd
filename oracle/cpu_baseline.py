"""CPU baseline for bench.py: the reference's loop structure on host cores.  TEST INFRASTRUCTURE.

The reference itself (Python highway-env + ppo/agent.py) cannot travel to the GPU box, so the
timed "reference CPU path" is a restatement with the reference's structure
(training/routine.py:121-243, ppo/agent.py:196-308):
  * one env per process (the C oracle, hwy_oracle.c, E = 1), OMP_NUM_THREADS = 1 per process
    (slurm_jobs/experiments_array.slurm.j2:21);
  * batch-1 actor-critic forward + sampling per step in torch on the CPU;
  * every `steps_per_update` steps, GAE (float64 loop as ppo/agent.py:126-138) and the clipped
    PPO update with one minibatch partition reused for all epochs, Adam, grad-clip.
P processes run side by side; the aggregate env-steps/s is their sum.  Python highway-env is
slower than the C oracle, so this baseline is optimistic for the reference.
"""

from __future__ import annotations

import multiprocessing as mp
import os
import sys
import time

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))


def _worker(args):
    seed, steps, steps_per_update, hidden, epochs, batch_size, lr, q = args
    os.environ["OMP_NUM_THREADS"] = "1"
    import torch
    import torch.nn as nn
    from torch.distributions import Normal

    torch.set_num_threads(1)
    sys.path.insert(0, os.path.dirname(_HERE))
    sys.path.insert(0, os.path.join(os.path.dirname(_HERE), "highway-rope-ppo_amd"))
    from oracle.oracle import OracleEnv
    from hwy._abi import config_from_dict
    from config.base_config import HIGHWAY_CONFIG

    cfg = config_from_dict(HIGHWAY_CONFIG, num_envs=1, autoreset=True, seed_base=seed)
    env = OracleEnv(cfg)
    sd = cfg.obs_vehicles * cfg.obs_features()

    class AC(nn.Module):
        def __init__(self):
            super().__init__()
            self.shared = nn.Sequential(nn.Linear(sd, hidden), nn.ReLU(), nn.Linear(hidden, hidden), nn.ReLU())
            self.actor_mean = nn.Sequential(nn.Linear(hidden, hidden), nn.ReLU(), nn.Linear(hidden, 2))
            self.log_std = nn.Parameter(torch.zeros(2))
            self.critic = nn.Sequential(nn.Linear(hidden, hidden), nn.ReLU(), nn.Linear(hidden, 1))

        def forward(self, x):
            h = self.shared(x)
            return self.actor_mean(h), self.log_std.exp(), self.critic(h)

    torch.manual_seed(seed)
    np.random.seed(seed)
    ac = AC()
    opt = torch.optim.Adam(ac.parameters(), lr=lr)
    obs = env.reset()
    S, Z, LP, R, D, V = [], [], [], [], [], []
    done_steps = 0
    t0 = time.perf_counter()
    while done_steps < steps:
        x = torch.as_tensor(obs.reshape(-1))
        with torch.no_grad():
            m, s, v = ac(x)
            dist = Normal(m, s)
            z = dist.sample()
            a = torch.tanh(z)
            lp = (dist.log_prob(z) - torch.log1p(-a.pow(2) + 1e-6)).sum(-1)
        obs, r, te, tr, _, _ = env.step(a.numpy()[None])
        S.append(x.numpy())
        Z.append(z.numpy())
        LP.append(float(lp))
        R.append(float(r[0]))
        D.append(bool(te[0] or tr[0]))
        V.append(float(v[0]))
        done_steps += 1
        if len(S) == steps_per_update or done_steps == steps:
            with torch.no_grad():
                last = 0.0 if D[-1] else float(ac(torch.as_tensor(obs.reshape(-1)))[2][0])
            vals = np.array(V + [last])
            adv = np.zeros(len(R), np.float32)
            la = 0.0
            for t in reversed(range(len(R))):
                nd = 1.0 - D[t]
                delta = R[t] + 0.99 * vals[t + 1] * nd - vals[t]
                adv[t] = delta + 0.99 * 0.95 * nd * la
                la = adv[t]
            ret = torch.as_tensor(adv + np.array(V, np.float32))
            advt = torch.as_tensor(adv)
            advt = (advt - advt.mean()) / (advt.std() + 1e-8)
            st, zt, lpt = torch.as_tensor(np.array(S)), torch.as_tensor(np.array(Z)), torch.as_tensor(LP, dtype=torch.float32)
            idx = np.arange(len(S))
            np.random.shuffle(idx)
            for _ in range(epochs):
                for i in range(0, len(S), batch_size):
                    b = torch.as_tensor(idx[i:i + batch_size])
                    m, s, v = ac(st[b])
                    dist = Normal(m, s)
                    zz = zt[b]
                    nlp = (dist.log_prob(zz) - torch.log1p(-torch.tanh(zz).pow(2) + 1e-6)).sum(-1)
                    ratio = torch.exp(nlp - lpt[b])
                    s1, s2 = ratio * advt[b], torch.clamp(ratio, 0.8, 1.2) * advt[b]
                    loss = (-torch.min(s1, s2).mean() + 0.5 * ((v.squeeze(-1) - ret[b]) ** 2).mean()
                            - 0.005 * dist.entropy().sum(-1).mean())
                    opt.zero_grad()
                    loss.backward()
                    nn.utils.clip_grad_norm_(ac.parameters(), 0.5)
                    opt.step()
            S, Z, LP, R, D, V = [], [], [], [], [], []
    dt = time.perf_counter() - t0
    q.put((done_steps, dt))


def run(procs: int = 4, steps: int = 2048, steps_per_update: int = 2048, hidden: int = 256,
        epochs: int = 8, batch_size: int = 64, lr: float = 3e-4) -> dict:
    """Time `procs` independent reference-structure training processes; returns a summary."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=((42 + 1000 * i, steps, steps_per_update, hidden, epochs,
                                            batch_size, lr, q),)) for i in range(procs)]
    for p in ps:
        p.start()
    res = [q.get() for _ in ps]
    for p in ps:
        p.join()
    per_proc = [s / t for s, t in res]
    return {
        "value": float(sum(per_proc)),
        "per_core": float(np.mean(per_proc)),
        "cores": procs,
        "seconds": float(max(t for _, t in res)),
        "steps_per_proc": steps,
    }


if __name__ == "__main__":
    print(run(procs=int(sys.argv[1]) if len(sys.argv) > 1 else 2,
              steps=int(sys.argv[2]) if len(sys.argv) > 2 else 2048))
