#!/usr/bin/env python3
"""stats.json for a recipe run directory (summary.jsonl from tools/train_parity.py): mean / std
of final_reward over seeds, the reference's matched seeds (42/1042/2042) beside the reference's
values, env-steps and wall-clock per run, and the env-steps at which the moving average of the
last 10 evals (routine.py's avg_rewards) first reaches the target band (132.42 - 5)."""

import json
import sys

import numpy as np

REF = {42: 136.8270, 1042: 127.8022, 2042: 132.6172}  # artifacts/combined_validated_data-final-run.csv


def main(d, note=""):
    global REF
    rows = [json.loads(l) for l in open(f"{d}/summary.jsonl")]
    # the run's own reference cell when the summary carries it (PE conditions, hidden sweep)
    own = {r["seed"]: r["reference_final_reward"] for r in rows if "reference_final_reward" in r}
    if own:
        REF = own
    fr = np.array([r["final_reward"] for r in rows])
    out = {"note": note, "condition": rows[0].get("condition"),
           "hidden_dim": rows[0].get("hidden_dim", 256), "n": len(rows), "mean": round(float(fr.mean()), 2),
           "std": round(float(fr.std()), 2), "min": float(fr.min()), "max": float(fr.max()),
           "reference_mean_3seeds": round(float(np.mean(list(REF.values()))), 2), "per_seed": []}
    m3 = [r["final_reward"] for r in rows if r["seed"] in REF]
    if m3:
        out["matched_seeds_mean"] = round(float(np.mean(m3)), 2)
        ref_mean = float(np.mean(list(REF.values())))
        out["matched_delta"] = round(out["matched_seeds_mean"] - ref_mean, 2)
        out["matched_in_band"] = bool(abs(out["matched_seeds_mean"] - ref_mean) <= 5.0)
        out["mean_in_band"] = bool(abs(float(fr.mean()) - ref_mean) <= 5.0)
    band = np.mean(list(REF.values())) - 5.0
    for r in rows:
        ev = np.array(r["evals"])
        eps = np.array(r["eval_episodes"])
        avg = np.array([ev[max(0, i - 9):i + 1].mean() for i in range(len(ev))])
        hit = np.nonzero((avg >= band) & (np.arange(len(ev)) >= 9))[0]
        steps_per_ep = r["env_steps"] / max(1, r["episodes"])
        out["per_seed"].append({
            "seed": r["seed"], "final_reward": r["final_reward"], "reference": REF.get(r["seed"]),
            "env_steps": r["env_steps"], "updates": r["updates"], "train_s": r["train_s"],
            "wall_s": r["wall_s"],
            "episodes_to_band": int(eps[hit[0]]) if hit.size else None,
            "approx_env_steps_to_band": int(eps[hit[0]] * steps_per_ep) if hit.size else None})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
