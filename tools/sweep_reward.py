#!/usr/bin/env python3
"""The condition sweep at the reference's own update statistics, run as grouped experiments.

For each of the six reference cells (sorted h256 / h384 / h512, shuffled RoPE / DistPE / RankPE
h256, d_embed 4) the seeds 42, 1042, ..., 9042 run as ONE ExperimentRunner.launch_group call
(experiments/runner.py -> ppo/group.py: the seeds batched into the env, acting and minibatch-step
launches, each bit-identical to its solo launch()), at the recipe of tools/train_parity.py
--num-envs 16 --rollout 128 --minibatches 32 --episodes 1500 --eval-interval 50 (the reference's
2,048 samples per update in minibatches of 64, 8 epochs, lr 3e-4).

Each cell writes OUT/<condition>_h<H>_e<E>_t<T>/summary.jsonl (the layout tools/recipe_stats.py
and tools/condition_order.py read; run them afterwards -- no child process is started from this
GPU process).  Each run's final_reward is compared with the solo runs of the same recipe and seed recorded in
round 4 (profiles/r4/reward/<cell>_e16_t128/summary.jsonl, one ExperimentRunner.launch per
process-sequential run): every kernel change since is bit-identical, so the grouped sweep must
reproduce them exactly.  Also writes OUT/sweep.json (wall time, per-cell agreement) and prints
one line per cell.

    python tools/sweep_reward.py --out gpurun_out/sweep_reward [--cells sorted_h256 ...]
        [--seeds 42 1042 ...] [--work /tmp/sweep_work] [--batch]
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "highway-rope-ppo_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

CELLS = {"sorted_h256": ("sorted", 256), "sorted_h384": ("sorted", 384),
         "sorted_h512": ("sorted", 512), "shuffled_rope_h256": ("shuffled_rope", 256),
         "shuffled_distpe_h256": ("shuffled_distpe", 256),
         "shuffled_rankpe_h256": ("shuffled_rankpe", 256)}


def _write_cell(out, cell, exps, results, wall, unit_cells, E, T, M, args, reference_final):
    """summary.jsonl of one cell (tools/condition_order.py layout) and its report entry."""
    cname, H = CELLS[cell]
    d_embed = None if cname == "sorted" else 4
    run_dir = os.path.join(out, f"{cname}_h{H}_e{E}_t{T}")
    os.makedirs(run_dir, exist_ok=True)
    solo = {}
    solo_path = os.path.join(ROOT, "profiles", "r4", "reward", f"{cell}_e{E}_t{T}",
                             "summary.jsonl")
    if os.path.exists(solo_path):
        for line in open(solo_path):
            r = json.loads(line)
            if r.get("episodes") == args.episodes and r.get("eval_interval") == args.eval_interval:
                solo[int(r["seed"])] = r.get("final_reward")
    rows, same = [], []
    ref = reference_final(cname, H)
    with open(os.path.join(run_dir, "summary.jsonl"), "w") as f:
        for e, res in zip(exps, results):
            row = {"condition": cname, "seed": e.seed, "experiment": e.name,
                   "status": res["status"], "num_envs": E, "episodes": args.episodes,
                   "rollout": T, "minibatches": M, "eval_interval": args.eval_interval,
                   "lr": 3e-4, "epochs": 8, "hidden_dim": H, "obs_vehicles": 15,
                   "order": "make_env default", "d_embed": d_embed, "grouped": len(exps),
                   "cells_in_batch": unit_cells}
            if res["status"] == "COMPLETED":
                avg = res["avg_rewards"]
                hist = res["metrics_history"]
                ups = hist.get("policy_updates", [])
                row.update(final_reward=round(float(avg[-1]), 4),
                           max_reward=round(float(max(avg)), 4),
                           evals=[round(float(x), 2) for x in hist.get("eval_rewards", [])],
                           eval_episodes=[int(x) for x in hist.get("eval_episode_numbers", [])],
                           env_steps=int(sum(u.get("steps", 0) for u in ups)),
                           updates=len(ups),
                           # the group's (or batch's) wall clock, shared by its experiments
                           wall_s=round(wall, 1), train_s=round(wall, 1))
                if e.seed in ref:
                    row.update(reference_final_reward=ref[e.seed],
                               delta=round(row["final_reward"] - ref[e.seed], 4))
                if e.seed in solo:
                    row["solo_r4_final_reward"] = solo[e.seed]
                    same.append(row["final_reward"] == solo[e.seed])
            else:
                row["error"] = res.get("error_message")
            rows.append(row)
            f.write(json.dumps(row) + "\n")
    done = [r["final_reward"] for r in rows if "final_reward" in r]
    return {"wall_s": round(wall, 1), "n": len(done),
            "mean_final_reward": round(sum(done) / len(done), 4) if done else None,
            "equal_to_solo_r4": f"{sum(same)}/{len(same)}" if same else None,
            "env_steps": int(sum(r.get("env_steps", 0) for r in rows)),
            "cells_in_batch": unit_cells}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--out", default="gpurun_out/sweep_reward")
    p.add_argument("--work", default=None,
                   help="where the runner writes each cell's logs, checkpoints and artifacts "
                        "(default: the cell's directory under --out); the summaries always go "
                        "under --out")
    p.add_argument("--cells", nargs="+", default=list(CELLS))
    p.add_argument("--seeds", type=int, nargs="+", default=[42 + 1000 * k for k in range(10)])
    p.add_argument("--episodes", type=int, default=1500)
    p.add_argument("--num-envs", type=int, default=16)
    p.add_argument("--rollout", type=int, default=128)
    p.add_argument("--minibatches", type=int, default=32)
    p.add_argument("--eval-interval", type=int, default=50)
    p.add_argument("--batch", action="store_true",
                   help="run the cells of one hidden width as one ExperimentRunner.launch_batch "
                        "(one GroupBatch: shared acting, env and minibatch-step launches)")
    args = p.parse_args()
    out = os.path.abspath(args.out)
    os.makedirs(out, exist_ok=True)

    from config.base_config import HIGHWAY_CONFIG
    from experiments.config import Condition, ConditionHP, Experiment
    from experiments.runner import ExperimentRunner
    from train_parity import reference_final

    conds = {"sorted": Condition.SORTED, "shuffled_rope": Condition.SHUFFLED_ROPE,
             "shuffled_distpe": Condition.SHUFFLED_DISTPE,
             "shuffled_rankpe": Condition.SHUFFLED_RANKPE}
    E, T, M = args.num_envs, args.rollout, args.minibatches
    report = {"recipe": {"num_envs": E, "rollout": T, "minibatches": M, "episodes": args.episodes,
                         "eval_interval": args.eval_interval, "seeds": args.seeds},
              "cells": {}}
    t_all = time.time()
    cell_exps = {}
    for cell in args.cells:
        cname, H = CELLS[cell]
        d_embed = None if cname == "sorted" else 4
        exps = []
        for seed in args.seeds:
            # tools/train_parity.py's experiment for this recipe and seed
            name = (f"{cname}_lr0.0003_hidden_dim{H}_clip_eps0.2_entropy_coef0.005_epochs8_"
                    "batch_size64" + (f"_d_embed{d_embed}" if d_embed else "")
                    + f"_seed{seed}_envs{E}_T{T}_mb{M}")
            hp = ConditionHP(lr=3e-4, clip_eps=0.2, epochs=8, batch_size=64, hidden_dim=H,
                             d_embed=d_embed)
            hp.entropy_coef = 0.005
            hp.steps_per_update = E * T
            extra = {"log_interval": max(50, args.episodes // 200),
                     "eval_interval": args.eval_interval, "num_envs": E, "num_minibatches": M}
            exps.append(Experiment(name=name, condition=conds[cname], hp=hp, seed=seed,
                                   max_episodes=args.episodes, target_reward=130.0, extra=extra,
                                   env_config_overrides={}))
        cell_exps[cell] = exps
    # execution units: one launch_group per cell, or (--batch) one launch_batch per hidden width
    if args.batch:
        by_h = {}
        for cell in args.cells:
            by_h.setdefault(CELLS[cell][1], []).append(cell)
        units = list(by_h.values())
    else:
        units = [[cell] for cell in args.cells]
    for unit in units:
        tag = unit[0] if len(unit) == 1 else "batch_h%d" % CELLS[unit[0]][1]
        work_dir = os.path.join(os.path.abspath(args.work) if args.work else out, tag)
        os.makedirs(work_dir, exist_ok=True)
        cwd = os.getcwd()
        os.chdir(work_dir)
        t0 = time.time()
        try:
            runner = ExperimentRunner(HIGHWAY_CONFIG)
            per_cell = (runner.launch_batch([cell_exps[c] for c in unit]) if len(unit) > 1
                        else [runner.launch_group(cell_exps[unit[0]])])
        finally:
            os.chdir(cwd)
        wall = time.time() - t0
        for cell, results in zip(unit, per_cell):
            report["cells"][cell] = _write_cell(out, cell, cell_exps[cell], results, wall,
                                                len(unit), E, T, M, args, reference_final)
            print(json.dumps({"cell": cell, **report["cells"][cell]}), flush=True)
    report["wall_s"] = round(time.time() - t_all, 1)
    with open(os.path.join(out, "sweep.json"), "w") as f:
        json.dump(report, f, indent=1)
    print(json.dumps({"total_wall_s": report["wall_s"]}), flush=True)


if __name__ == "__main__":
    main()
