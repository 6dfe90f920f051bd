#!/bin/bash
# compact-LDS ppo_rows: section clocks (profiling build) and a start-stagger sweep (dev build)
set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 120 python -u tools/probe_ppo_sections.py 256 16384 > gpurun_out/r3/sections_cmp.log 2>&1; rc=$?
cat gpurun_out/r3/sections_cmp.log; [ $rc -eq 0 ] || exit $rc
D=$PWD/highway-rope-ppo_amd/hwy/libhwy_dev.so
for st in 0 1 2 4 8 0 1 2 4 8; do
  HWY_LIB=$D HWY_ROWS_STAGGER=$st timeout -k 10 60 python -u tools/probe_ppo_time.py 256 10 16384 | sed "s/^/stagger=$st /" || exit 1
done
