"""Condition ordering of one reward recipe against the reference study.

Reads the six cells' stats.json of a recipe (tools/recipe_stats.py output) -- sorted h256 / h384 /
h512, shuffled_rope / shuffled_distpe / shuffled_rankpe h256 d_embed 4 -- and reports, beside
the reference's batch_size-64 means of the same cells: each cell's mean and 95 % CI, the order of
the cells on both sides, the Spearman rank correlation of the six means, and the one contrast the
reference study is about, sorted h256 against the three PE conditions (Welch's t on the seeds).

    python tools/condition_order.py DIR E T [--out FILE]
DIR holds <condition>_h<H>_e<E>_t<T>/stats.json (e.g. profiles/r5/reward).
"""

import argparse
import json
import math
import os

CELLS = [("sorted", 256), ("sorted", 384), ("sorted", 512), ("shuffled_rope", 256),
         ("shuffled_distpe", 256), ("shuffled_rankpe", 256)]


def _seeds(path):
    rows = [json.loads(l) for l in open(os.path.join(os.path.dirname(path), "summary.jsonl"))
            if l.strip()]
    return [r["final_reward"] for r in rows if r.get("status") == "COMPLETED"]


def _welch(a, b):
    na, nb = len(a), len(b)
    ma, mb = sum(a) / na, sum(b) / nb
    va = sum((x - ma) ** 2 for x in a) / (na - 1)
    vb = sum((x - mb) ** 2 for x in b) / (nb - 1)
    se = math.sqrt(va / na + vb / nb)
    t = (ma - mb) / se if se > 0 else float("inf")
    df = (va / na + vb / nb) ** 2 / ((va / na) ** 2 / (na - 1) + (vb / nb) ** 2 / (nb - 1))
    try:
        from scipy import stats

        p = float(2 * stats.t.sf(abs(t), df))
    except Exception:  # scipy absent: normal approximation
        p = float(math.erfc(abs(t) / math.sqrt(2)))
    return {"diff": round(ma - mb, 2), "t": round(t, 3), "df": round(df, 1), "p_two_sided": round(p, 4)}


def _ranks(v):
    order = sorted(range(len(v)), key=lambda i: -v[i])
    r = [0] * len(v)
    for k, i in enumerate(order):
        r[i] = k + 1
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("E", type=int)
    ap.add_argument("T", type=int)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    cells, ours, ref = [], [], []
    seeds = {}
    for cond, h in CELLS:
        path = os.path.join(a.dir, f"{cond}_h{h}_e{a.E}_t{a.T}", "stats.json")
        if not os.path.exists(path):
            continue
        st = json.load(open(path))
        seeds[(cond, h)] = _seeds(path)
        cells.append({"cell": f"{cond} h{h}", "mean": st["mean"], "sd": st["std"],
                      "ci95": (st.get("ours") or {}).get("ci95"), "n": st["n"],
                      "matched_seeds_mean": st.get("matched_seeds_mean"),
                      "reference_bs64_mean": st.get("reference_mean_3seeds"),
                      "delta": round(st["mean"] - st["reference_mean_3seeds"], 2)})
        ours.append(st["mean"])
        ref.append(st["reference_mean_3seeds"])
    out = {"recipe": {"E": a.E, "T": a.T}, "cells": cells}
    if len(cells) >= 2:
        ro, rr = _ranks(ours), _ranks(ref)
        n = len(cells)
        rho = 1 - 6 * sum((x - y) ** 2 for x, y in zip(ro, rr)) / (n * (n * n - 1))
        out["order_ours"] = [cells[i]["cell"] for i in sorted(range(n), key=lambda i: -ours[i])]
        out["order_reference"] = [cells[i]["cell"] for i in sorted(range(n), key=lambda i: -ref[i])]
        out["spearman_rho"] = round(rho, 3)
    s = seeds.get(("sorted", 256))
    if s:
        out["sorted_h256_vs_pe"] = {
            f"{c} h{h}": _welch(s, seeds[(c, h)])
            for c, h in CELLS[3:] if (c, h) in seeds}
        spread = [x["mean"] for x in cells]
        out["spread_of_means"] = round(max(spread) - min(spread), 2)
    txt = json.dumps(out, indent=1)
    print(txt)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main()
