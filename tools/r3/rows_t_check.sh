#!/bin/bash
# ppo_rowsT: the fused-gradient tests that select it, then A/B timing against ppo_rows (dev lib)
set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 400 python -u -m pytest tests/test_ppo_fused_gpu.py -x -v --timeout 200 --timeout-method thread \
  -k "16384 or 32768 or every_step or replays" > gpurun_out/r3/rows_t_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r3/rows_t_tests.log
[ $rc -eq 0 ] || exit $rc
D=$PWD/highway-rope-ppo_amd/hwy/libhwy_dev.so
for mb in 16384 32768; do
  for t in 1 0; do
    HWY_LIB=$D HWY_ROWS_T=$t timeout -k 10 60 python -u tools/probe_ppo_time.py 256 5 $mb | sed "s/^/rows_t=$t mb=$mb /" || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3/prof_rowsT -o run -- python3 tools/probe_ppo_time.py 256 3 16384 > gpurun_out/r3/prof_rowsT.log 2>&1 || exit 1
f=$(find gpurun_out/r3/prof_rowsT -name "*kernel_stats.csv" | head -1); python3 tools/summarize_stats.py "$f" 12
