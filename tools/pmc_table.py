"""Per-kernel mean of every counter in rocprofv3 counter_collection CSVs under a directory."""
import collections, csv, glob, sys

root = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in agg.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:40s} {sum(v) / len(v):16,.0f}   (n={len(v)})")
