#!/usr/bin/env python3
"""Where a grouped sweep batch's iteration goes (development aid): the four h256 cells x G seeds
at E = 16, T = 128 as one GroupBatch (bench.py --sweep's largest batch), timed per part with a
device sync around each -- the rollout, the update (bootstrap act, each group's pre_update: GAE,
normalisation, permutation mapping; the grouped minibatch steps; post_update) -- and the
update's pre / steps / post split by host clock.

    python tools/probe_sweep_split.py [G]
"""

import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "highway-rope-ppo_amd"))

import torch  # noqa: E402


def main():
    from config.base_config import HIGHWAY_CONFIG
    from experiments.config import Condition
    from ppo.agent import PPOAgent
    from ppo.group import GroupBatch, _run_group_steps, build_group

    G = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    dev = torch.device("cuda", 0)
    seeds = [42 + 1000 * k for k in range(G)]
    groups = []
    for name, d in (("SORTED", None), ("SHUFFLED_ROPE", 4), ("SHUFFLED_DISTPE", 4),
                    ("SHUFFLED_RANKPE", 4)):
        groups.append(build_group(Condition[name], HIGHWAY_CONFIG, seeds, 16, 128, dev,
                                  lambda sd: PPOAgent(sd, 2, device=dev, lr=3e-4, epochs=8,
                                                      batch_size=64, hidden_dim=256),
                                  d_embed=d))
    b = GroupBatch(groups)
    for _ in range(3):
        b.iteration(return_metrics=True)
    torch.cuda.synchronize()
    sync = torch.cuda.synchronize
    acc = {"rollout": 0.0, "boot_act": 0.0, "pre_update": 0.0, "steps": 0.0, "post_update": 0.0}
    n = 5
    for _ in range(n):
        t0 = time.perf_counter()
        b.rollout()
        sync()
        t1 = time.perf_counter()
        b.act.launch(b._rows(0, deterministic=True))
        sync()
        t2 = time.perf_counter()
        ctxs = [g.pre_update(g._boot[3]) for g in b.groups]
        sync()
        t3 = time.perf_counter()
        b._runner = _run_group_steps(b, ctxs, b._runner)
        sync()
        t4 = time.perf_counter()
        [g.post_update(c, True) for g, c in zip(b.groups, ctxs)]
        sync()
        t5 = time.perf_counter()
        for k, v in zip(acc, (t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4)):
            acc[k] += v
    tot = sum(acc.values())
    print(f"G={G} x 4 cells: {tot / n * 1e3:.2f} ms per iteration", flush=True)
    for k, v in acc.items():
        print(f"  {k:12s} {v / n * 1e3:8.2f} ms", flush=True)
    print("stats", b.stats, flush=True)


if __name__ == "__main__":
    main()
