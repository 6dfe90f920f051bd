"""Summarise a rocprofv3 --stats kernel CSV: top kernels by total time."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"{'total ms':>9} {'%':>6} {'calls':>7} {'avg us':>9}  kernel")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.2f} {float(r['Percentage']):6.2f} {r['Calls']:>7} "
          f"{float(r['AverageNs'])/1e3:9.2f}  {r['Name'][:100]}")
print(f"sum of kernel time: {tot/1e6:.1f} ms over {sum(int(r['Calls']) for r in rows)} launches")
