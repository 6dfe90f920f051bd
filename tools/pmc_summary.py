"""Average rocprofv3 --pmc counters per kernel (development aid): pmc_summary.py <dir> [filter]"""
import collections, csv, glob, sys

d = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{d}/**/*_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if flt in r["Kernel_Name"]:
            agg[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in agg.items():
    waves = sum(cs["SQ_WAVES"]) / len(cs["SQ_WAVES"]) if "SQ_WAVES" in cs else None
    print(k)
    for c, v in sorted(cs.items()):
        m = sum(v) / len(v)
        extra = f"  per-wave {m / waves:,.0f}" if waves and c != "SQ_WAVES" else ""
        print(f"  {c:24s} n={len(v):3d} mean={m:,.0f}{extra}")
