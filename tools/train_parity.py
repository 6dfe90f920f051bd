#!/usr/bin/env python3
"""Reward-parity training runs: the reference's north-star cell on the MI355X env.

Runs `ExperimentRunner.launch` (experiments/runner.py, the reference's runner sequence,
/root/reference/experiments/runner.py:73-122) for the reference experiment
`<condition>_lr0.0003_hidden_dim256_clip_eps0.2_entropy_coef0.005_epochs8_batch_size64` at the
given seeds, 1500 episodes, eval every 50 episodes, and compares `final_reward` (mean of the last 10
evals, each the mean of 5 deterministic episodes seeded exp_seed+1000+k;
training/routine.py:181-186,292) with the reference's published value for the same seed
(artifacts/combined_validated_data-final-run.csv rows sorted_..._hidden_dim256_..._batch_size64:
seed 42 136.8270, 1042 127.8022, 2042 132.6172; mean 132.42).

Usage (GPU box):  python tools/train_parity.py --seeds 42 --out gpurun_out/train
    --num-envs 1   the reference's own loop (1 env, batch-1 select_action, 2048-step updates)
    --num-envs E   the lockstep loop (E envs, same hyperparameters, same episode budget)
Under torchrun (--nproc-per-node N) each experiment spans the N GPUs with E envs per rank
(experiments/runner.py); rank 0 prints and writes the summary.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "highway-rope-ppo_amd"))

# artifacts/combined_validated_data-final-run.csv, lr 3e-4 / h256 / clip .2 / ent .005 / 8 epochs /
# bs 64 (d_embed 4 for the PE conditions; the reference's own DistPE and RoPE rows coincide)
REFERENCE_FINAL = {
    "sorted": {42: 136.8270, 1042: 127.8022, 2042: 132.6172},
    "shuffled_rope": {42: 136.0069, 1042: 82.4615, 2042: 125.5533},
    "shuffled_distpe": {42: 136.0069, 1042: 82.4615, 2042: 125.5533},
    "shuffled_rankpe": {42: 83.2977, 1042: 119.7457, 2042: 119.0862},
}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--seeds", type=int, nargs="+", default=[42])
    p.add_argument("--episodes", type=int, default=1500)
    p.add_argument("--num-envs", type=int, default=1)
    p.add_argument("--out", default="gpurun_out/train")
    p.add_argument("--condition", default="sorted", choices=sorted(REFERENCE_FINAL))
    args = p.parse_args()

    out = os.path.abspath(args.out)
    os.makedirs(out, exist_ok=True)
    import torch

    from config.base_config import HIGHWAY_CONFIG
    from experiments.config import Condition, ConditionHP, Experiment
    from experiments.runner import ExperimentRunner

    results = []
    cond = {"sorted": Condition.SORTED, "shuffled_rope": Condition.SHUFFLED_ROPE,
            "shuffled_distpe": Condition.SHUFFLED_DISTPE,
            "shuffled_rankpe": Condition.SHUFFLED_RANKPE}[args.condition]
    d_embed = None if args.condition == "sorted" else 4
    for seed in args.seeds:
        name = (f"{args.condition}_lr0.0003_hidden_dim256_clip_eps0.2_entropy_coef0.005_epochs8_"
                f"batch_size64" + (f"_d_embed{d_embed}" if d_embed else "") + f"_seed{seed}"
                + (f"_envs{args.num_envs}" if args.num_envs > 1 else ""))
        hp = ConditionHP(lr=3e-4, clip_eps=0.2, epochs=8, batch_size=64, hidden_dim=256,
                         d_embed=d_embed)
        hp.entropy_coef = 0.005
        extra = {"log_interval": 50, "eval_interval": 50}
        if args.num_envs > 1:
            extra["num_envs"] = args.num_envs
        exp = Experiment(name=name, condition=cond, hp=hp, seed=seed,
                         max_episodes=args.episodes, target_reward=130.0, extra=extra)
        run_dir = os.path.join(out, f"{args.condition}_seed{seed}")
        os.makedirs(run_dir, exist_ok=True)
        cwd = os.getcwd()
        os.chdir(run_dir)
        t0 = time.time()
        try:
            res = ExperimentRunner(HIGHWAY_CONFIG).launch(exp)
        finally:
            os.chdir(cwd)
        wall = time.time() - t0
        row = {"condition": args.condition, "seed": seed, "experiment": name, "status": res["status"], "wall_s": round(wall, 1),
               "num_envs": args.num_envs, "episodes": args.episodes,
               "device": torch.cuda.get_device_name(0) if torch.cuda.is_available() else "cpu"}
        if res["status"] == "COMPLETED":
            avg = res["avg_rewards"]
            hist = res["metrics_history"]
            row.update(final_reward=round(float(avg[-1]), 4), max_reward=round(float(max(avg)), 4),
                       evals=[round(float(x), 2) for x in hist.get("eval_rewards", [])])
            ref = REFERENCE_FINAL[args.condition].get(seed)
            if ref is not None:
                row.update(reference_final_reward=ref,
                           delta=round(float(avg[-1]) - ref, 4))
        else:
            row["error"] = res.get("error_message")
        if res.get("rank", 0) != 0:
            continue
        row["world_size"] = int(os.environ.get("WORLD_SIZE", "1"))
        results.append(row)
        print(json.dumps(row), flush=True)
        with open(os.path.join(out, "summary.jsonl"), "a") as f:
            f.write(json.dumps(row) + "\n")
    done = [r for r in results if "final_reward" in r]
    if done:
        mean = sum(r["final_reward"] for r in done) / len(done)
        refs = [REFERENCE_FINAL[args.condition][r["seed"]] for r in done
                if r["seed"] in REFERENCE_FINAL[args.condition]]
        print(json.dumps({"condition": args.condition, "mean_final_reward": round(mean, 4),
                          "reference_mean": round(sum(refs) / len(refs), 4) if refs else None,
                          "n": len(done)}), flush=True)


if __name__ == "__main__":
    main()
