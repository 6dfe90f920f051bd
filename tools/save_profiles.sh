#!/bin/bash
# Copy the judged artefacts of the last tools/gpu_check.sh run from gpurun_out/ into profiles/r1/.
set -e
D=profiles/r1
grep '^{' gpurun_out/bench.log > $D/bench_latest.json
grep '^{' gpurun_out/bench_prof.log > $D/bench_under_rocprof.log
cp gpurun_out/gpu_tests.log $D/gpu_tests.log
S=$(ls gpurun_out/prof/run_kernel_stats.csv gpurun_out/prof/*/run_kernel_stats.csv 2>/dev/null | head -1)
python3 tools/summarize_stats.py "$S" 14 > $D/bench_kernel_stats_top.txt
cp "$S" $D/bench_kernel_stats.csv
