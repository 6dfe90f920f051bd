#!/bin/bash
# GPU test suite + smoke + default bench on the box (each step time-limited, chained with &&)
set -o pipefail
mkdir -p gpurun_out/r4
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r4/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r4/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4/smoke.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/r4/bench_c1.json 2> gpurun_out/r4/bench_c1.err && \
cut -c1-400 gpurun_out/r4/bench_c1.json
