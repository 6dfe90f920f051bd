#!/bin/bash
# SQ instruction counts per hwy_step launch, product vs variants ($VARS), configs[1] shape
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/pmcab
for lib in libhwy.so $(for v in $VARS; do echo libhwy_$v.so; done); do
  d=$R/gpurun_out/pmcab/${lib%.so}
  HWY_LIB=$R/highway-rope-ppo_amd/hwy/$lib timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_WAVES \
    --kernel-include-regex hwy_step -d $d -o run --output-format csv -- python3 $R/tools/probe_step.py 4096 > $d.log 2>&1 || { echo "pmc $lib failed"; tail -3 $d.log; exit 1; }
  f=$(find $d -name "*counter_collection.csv" | head -1)
  python3 - "$f" "$lib" <<'PY'
import csv, sys
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    acc[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
n = len(acc)
keys = ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_BRANCH", "SQ_INSTS_LDS", "SQ_WAVES"]
avg = {k: sum(a[k] for a in acc.values()) / n for k in keys}
print(sys.argv[2], f"{n} launches;", " ".join(f"{k[9:]} {avg[k]/1e6:.2f}M" for k in keys))
PY
done
