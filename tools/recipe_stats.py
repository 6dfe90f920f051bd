#!/usr/bin/env python3
"""stats.json for a recipe run directory (summary.jsonl from tools/train_parity.py, or several
directories of one recipe merged): final_reward over seeds with its 95 % confidence interval, the
reference's matched seeds (42/1042/2042) beside the reference's values, the reference cell's own
spread (its 3 batch_size-64 seeds and its 3 batch_size-32 seeds, tools/reference_cells.py), a
Welch two-sample test of the difference, a TOST equivalence test against the +-5 band, env-steps
and wall-clock per run, and the env-steps at which the moving average of the last 10 evals
(routine.py's avg_rewards) first reaches the band's lower edge.

    python tools/recipe_stats.py DIR [DIR ...] [--note TEXT]
"""

import argparse
import json
import os
import sys

import numpy as np
from scipy import stats

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from reference_cells import REFERENCE  # noqa: E402

BAND = 5.0


def describe(x):
    x = np.asarray(x, np.float64)
    n = len(x)
    out = {"n": n, "mean": round(float(x.mean()), 2)}
    if n > 1:
        sd = float(x.std(ddof=1))
        half = float(stats.t.ppf(0.975, n - 1)) * sd / np.sqrt(n)
        out.update(sd=round(sd, 2), ci95=[round(float(x.mean()) - half, 2),
                                          round(float(x.mean()) + half, 2)])
    return out


def welch(a, b):
    """Welch's unequal-variance t-test of mean(a) - mean(b): t, df, two-sided p, the 95 % CI
    of the difference, and the TOST p-value for |difference| < BAND (equivalence is shown at the
    5 % level when it is below 0.05)."""
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    va, vb = a.var(ddof=1) / len(a), b.var(ddof=1) / len(b)
    se = float(np.sqrt(va + vb))
    df = float((va + vb) ** 2 / (va ** 2 / (len(a) - 1) + vb ** 2 / (len(b) - 1)))
    d = float(a.mean() - b.mean())
    t = d / se
    p = float(2 * stats.t.sf(abs(t), df))
    half = float(stats.t.ppf(0.975, df)) * se
    p_lo = float(stats.t.sf((d + BAND) / se, df))   # H0: d <= -BAND
    p_hi = float(stats.t.cdf((d - BAND) / se, df))  # H0: d >= +BAND
    return {"diff": round(d, 2), "t": round(t, 3), "df": round(df, 2), "p_two_sided": round(p, 4),
            "diff_ci95": [round(d - half, 2), round(d + half, 2)],
            "tost_p_within_band": round(max(p_lo, p_hi), 4),
            "significant_at_0.05": p < 0.05, "equivalent_within_band_at_0.05": max(p_lo, p_hi) < 0.05}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--note", default="")
    args = ap.parse_args()
    rows, seen = [], set()
    for d in args.dirs:
        for line in open(os.path.join(d, "summary.jsonl")):
            r = json.loads(line)
            if "final_reward" in r and r["seed"] not in seen:
                seen.add(r["seed"])
                rows.append(r)
    rows.sort(key=lambda r: r["seed"])
    cond = rows[0].get("condition", "sorted")
    hidden = rows[0].get("hidden_dim", 256)
    ref = REFERENCE.get((cond, hidden), {})
    r64 = ref.get("bs64", {})
    r32 = ref.get("bs32", {})
    fr = np.array([r["final_reward"] for r in rows])
    out = {"note": args.note, "condition": cond, "hidden_dim": hidden,
           "recipe": {k: rows[0].get(k) for k in ("num_envs", "rollout", "minibatches", "episodes",
                                                  "obs_vehicles", "order", "d_embed", "epochs",
                                                  "lr", "world_size")},
           "n": len(rows), "mean": round(float(fr.mean()), 2),
           "std": round(float(fr.std(ddof=1)), 2) if len(fr) > 1 else None,
           "min": float(fr.min()), "max": float(fr.max()), "ours": describe(fr)}
    if r64:
        ref_mean = float(np.mean(list(r64.values())))
        out["reference_mean_3seeds"] = round(ref_mean, 2)
        out["reference"] = {
            "source": "artifacts/combined_validated_data-final-run.csv (tools/reference_cells.py)",
            "bs64_seeds": r64, "bs64": describe(list(r64.values())),
            "bs32_seeds": r32, "bs32": describe(list(r32.values())) if r32 else None,
            "bs64_and_bs32": describe(list(r64.values()) + list(r32.values())) if r32 else None}
        m3 = [r for r in rows if r["seed"] in r64]
        if m3:
            ours3 = np.array([r["final_reward"] for r in m3])
            theirs3 = np.array([r64[r["seed"]] for r in m3])
            out["matched_seeds"] = [r["seed"] for r in m3]
            out["matched_seeds_mean"] = round(float(ours3.mean()), 2)
            out["matched_delta"] = round(float(ours3.mean() - theirs3.mean()), 2)
            out["matched_in_band"] = bool(abs(ours3.mean() - theirs3.mean()) <= BAND)
        out["mean_in_band"] = bool(abs(float(fr.mean()) - ref_mean) <= BAND)
        if len(fr) > 1:
            out["test_vs_reference_bs64"] = welch(fr, list(r64.values()))
            if r32:
                out["test_vs_reference_bs64_and_bs32"] = welch(fr, list(r64.values()) + list(r32.values()))
        out["band"] = BAND
        band_lo = ref_mean - BAND
    else:
        band_lo = None
    out["per_seed"] = []
    for r in rows:
        ev = np.array(r["evals"])
        eps = np.array(r["eval_episodes"])
        avg = np.array([ev[max(0, i - 9):i + 1].mean() for i in range(len(ev))])
        hit = (np.nonzero((avg >= band_lo) & (np.arange(len(ev)) >= 9))[0]
               if band_lo is not None else np.array([], int))
        steps_per_ep = r["env_steps"] / max(1, r["episodes"])
        out["per_seed"].append({
            "seed": r["seed"], "final_reward": r["final_reward"], "reference": r64.get(r["seed"]),
            "env_steps": r["env_steps"], "updates": r["updates"], "train_s": r["train_s"],
            "wall_s": r["wall_s"],
            "episodes_to_band": int(eps[hit[0]]) if hit.size else None,
            "approx_env_steps_to_band": int(eps[hit[0]] * steps_per_ep) if hit.size else None})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
