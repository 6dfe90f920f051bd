"""Calibrated hwy_step HBM bytes per launch from the pmc_step.sh passes
    python3 tools/calib/pmc_summarize.py <dir> [E N F_out]
-> profiles/hwy_step_pmc.json (E 4096, N 15, F_out 4) or profiles/hwy_step_pmc_E<E>_N<N>_F<F>.json"""
import csv
import re, glob, json, os, sys

d = sys.argv[1]
E = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
N = int(sys.argv[3]) if len(sys.argv) > 3 else 15
Fo = int(sys.argv[4]) if len(sys.argv) > 4 else 4
NF = 13
calib_bytes = NF * E * 64 * 4


def per_kernel(pass_dir, counter):
    out = {}
    for f in glob.glob(f"{pass_dir}/**/*_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            # "void hwy_step_kernel<4>(StepParams)" -> "hwy_step_kernel"
            name = re.sub(r"<.*>", "", r["Kernel_Name"].split("(")[0]).replace("void ", "").strip()
            out.setdefault(name, []).append(float(r["Counter_Value"]) * 1024.0)  # KiB -> B
    return {k: sum(v[1:]) / max(1, len(v) - 1) if len(v) > 1 else v[0] for k, v in out.items()}


fetch = per_kernel(f"{d}/fetch", "FETCH_SIZE")
write = per_kernel(f"{d}/write", "WRITE_SIZE")
kf = calib_bytes / fetch["calib_read"]
kw = calib_bytes / write["calib_write"]
step_read = fetch["hwy_step_kernel"] * kf
step_write = write["hwy_step_kernel"] * kw
res = {
    "kernel": "hwy_step_kernel", "envs_per_launch": E, "obs_rows": N, "obs_features": Fo,
    "fetch_size_raw_bytes": fetch["hwy_step_kernel"], "write_size_raw_bytes": write["hwy_step_kernel"],
    "calib_read_raw_bytes": fetch["calib_read"], "calib_write_raw_bytes": write["calib_write"],
    "calib_true_bytes": calib_bytes, "fetch_scale": kf, "write_scale": kw,
    "hbm_read_bytes_per_launch": step_read, "hbm_write_bytes_per_launch": step_write,
    "hbm_bytes_per_launch": step_read + step_write,
    "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; each scaled by "
              "true/measured bytes of calibration kernels with the same 4-B-lane, 256-B-row pattern",
}
print(json.dumps(res, indent=1))
os.makedirs("profiles", exist_ok=True)
out = ("profiles/hwy_step_pmc.json" if (E, N, Fo) == (4096, 15, 4)
       else f"profiles/hwy_step_pmc_E{E}_N{N}_F{Fo}.json")
json.dump(res, open(out, "w"), indent=1)
