#!/bin/bash
# A/B of the pre-gathered minibatch rows (FusedPPO.pregather): step time and per-kernel averages
set -o pipefail
OUT=gpurun_out/ab_pg; mkdir -p $OUT; R=$(pwd)
for rep in 1 2 3; do
  for pg in 1 0; do
    for mb in 4096 16384; do
      HWY_PREGATHER=$pg timeout -k 10 90 python -u tools/probe_ppo_time.py 256 10 $mb 60 | sed "s/^/pg=$pg mb=$mb /" || exit 1
    done
  done
done
cd /tmp && export TMPDIR=/tmp
for pg in 1 0; do
  d=$OUT/kt_pg$pg
  HWY_PREGATHER=$pg timeout -s KILL 120 rocprofv3 --kernel-trace --stats --kernel-include-regex "ppo_" \
    -d $d -o run --output-format csv -- python3 $R/tools/probe_ppo_time.py 256 3 4096 > $d.log 2>&1 || { echo "kt failed"; tail -3 $d.log; exit 1; }
  echo "== pregather $pg (4096 rows)"
  python3 $R/tools/summarize_stats.py "$(find $d -name '*kernel_stats.csv' | head -1)" 6
done
# then the first cells of the pre-registered intermediate recipe (profiles/r5/reward/PREREGISTERED.md)
cd $R
PART=B CELLS="sorted:256" bash tools/r5/reward_r5.sh
