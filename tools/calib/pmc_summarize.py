"""Calibrated hwy_step HBM bytes per launch from the pmc_step.sh passes -> profiles/hwy_step_pmc.json"""
import csv, glob, json, os, sys

d = sys.argv[1]
E, NF = 4096, 13
calib_bytes = NF * E * 64 * 4


def per_kernel(pass_dir, counter):
    out = {}
    for f in glob.glob(f"{pass_dir}/**/*_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            name = r["Kernel_Name"].split("(")[0]
            out.setdefault(name, []).append(float(r["Counter_Value"]) * 1024.0)  # KiB -> B
    return {k: sum(v[1:]) / max(1, len(v) - 1) if len(v) > 1 else v[0] for k, v in out.items()}


fetch = per_kernel(f"{d}/fetch", "FETCH_SIZE")
write = per_kernel(f"{d}/write", "WRITE_SIZE")
kf = calib_bytes / fetch["calib_read"]
kw = calib_bytes / write["calib_write"]
step_read = fetch["hwy_step_kernel"] * kf
step_write = write["hwy_step_kernel"] * kw
res = {
    "kernel": "hwy_step_kernel", "envs_per_launch": E,
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
json.dump(res, open("profiles/hwy_step_pmc.json", "w"), indent=1)
