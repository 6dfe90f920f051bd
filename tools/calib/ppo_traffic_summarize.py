"""Per-minibatch-step HBM-side traffic of the fused PPO update from tools/pmc_ppo_traffic.sh
    python3 tools/calib/ppo_traffic_summarize.py gpurun_out/pmc_ppo [rows]
        -> profiles/ppo_step_pmc.json (4096 rows) or profiles/ppo_step_pmc_<rows>.json

FETCH_SIZE / WRITE_SIZE count the L2's memory-side requests (Infinity-Cache hits included).
On gfx950 FETCH_SIZE reports half the bytes of 16-B-per-lane streaming reads, which is how
these kernels read (float4 rows, tile-image blocks), so reads are doubled; WRITE_SIZE is exact
for 16-B stores (MI355X_MICROARCH.md, HBM section).  ppo_wsum's scattered 4-B gradient stores
are uncalibrated (0.85 MB of the step's writes)."""
import collections, csv, glob, json, os, sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_ppo"
rows = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
S = int(sys.argv[3]) if len(sys.argv) > 3 else 60
H = int(sys.argv[4]) if len(sys.argv) > 4 else 256
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        for k in ("ppo_rows", "ppo_wgrad", "ppo_wsum", "ppo_adam"):
            if k in name:
                agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
per = {}
for k, cs in agg.items():
    fetch = sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"]) * 1024  # rocprofv3 reports KB
    write = sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"]) * 1024
    per[k] = {"fetch_size_raw_bytes": fetch, "write_size_raw_bytes": write,
              "read_bytes": 2 * fetch, "write_bytes": write, "launches": len(cs["FETCH_SIZE"])}
tot = sum(v["read_bytes"] + v["write_bytes"] for v in per.values())
res = {"kernel": f"PPO minibatch step ({rows} rows, S={S}, H={H})", "rows": rows, "S": S, "H": H,
       "per_kernel": per,
       "hbm_side_bytes_per_step": tot,
       "method": ("rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over "
                  "tools/probe_ppo_time.py <H> 2 <rows> <S> (tools/pmc_ppo_traffic.sh); FETCH_SIZE x2 for "
                  "16-B-per-lane reads, WRITE_SIZE as is; counts L2 memory-side requests, so "
                  "Infinity-Cache hits are included")}
os.makedirs("profiles", exist_ok=True)
if (S, H) == (60, 256):
    out = "profiles/ppo_step_pmc.json" if rows == 4096 else f"profiles/ppo_step_pmc_{rows}.json"
else:
    out = f"profiles/ppo_step_pmc_{rows}_S{S}_H{H}.json"
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
