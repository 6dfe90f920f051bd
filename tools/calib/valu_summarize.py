"""hwy_step instruction counts per launch from a PMC run -> profiles/hwy_step_valu.json
    python3 tools/calib/valu_summarize.py gpurun_out/pmck [N F_out]
(E 4096, N 15, F_out 4 -> profiles/hwy_step_valu.json; else hwy_step_valu_E<E>_N<N>_F<F>.json)"""
import collections, csv, glob, json, sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmck"
N = int(sys.argv[2]) if len(sys.argv) > 2 else 15
Fo = int(sys.argv[3]) if len(sys.argv) > 3 else 4
agg = collections.defaultdict(list)
names = set()
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "hwy_step" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
            names.add(r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0].strip())
m = {k: sum(v) / len(v) for k, v in agg.items()}
E = int(round(m["SQ_WAVES"]))
res = {"kernel": " + ".join(sorted(names)), "envs_per_launch": E, "obs_rows": N, "obs_features": Fo,
       "valu_insts_per_launch": m["SQ_INSTS_VALU"], "salu_insts_per_launch": m["SQ_INSTS_SALU"],
       "lds_insts_per_launch": m["SQ_INSTS_LDS"], "branch_insts_per_launch": m["SQ_INSTS_BRANCH"],
       "waves_per_launch": m["SQ_WAVES"], "valu_insts_per_wave": m["SQ_INSTS_VALU"] / m["SQ_WAVES"],
       "valu_issue_peak_per_s": 256 * 4 * 0.5 * 2.4e9,
       "method": ("rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVES "
                  "(tools/pmc_kernel.sh hwy_step step python3 tools/probe_step.py 4096; this script); "
                  "peak = 256 CUs x 4 SIMDs x one wave64 VALU instruction per 2 cycles x 2.4 GHz "
                  "(MI355X_MICROARCH.md: v_fma_f32 wave64 2 cyc per SIMD)")}
out = ("profiles/hwy_step_valu.json" if (E, N, Fo) == (4096, 15, 4)
       else f"profiles/hwy_step_valu_E{E}_N{N}_F{Fo}.json")
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
