#!/usr/bin/env python3
"""Average SQ counters per dispatch from a rocprofv3 counter_collection.csv (tools/ab.sh MODE=pmc)."""
import csv
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    acc[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
n = len(acc)
keys = sorted({k for a in acc.values() for k in a})
avg = {k: sum(a.get(k, 0.0) for a in acc.values()) / n for k in keys}
print(sys.argv[2] if len(sys.argv) > 2 else "", f"{n} launches;",
      " ".join(f"{k.replace('SQ_INSTS_', '')} {avg[k] / 1e6:.3f}M" for k in keys))
