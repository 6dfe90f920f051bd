#!/bin/bash
# GPU tests, then the bench for configs 1 (with the CPU baseline) and 2 / 3 / 4.
set -u
OUT=${OUT:-gpurun_out/r2c}
mkdir -p "$OUT"
{ nproc; python -c "import os;print('cpu_count', os.cpu_count(), 'affinity', len(os.sched_getaffinity(0)))";
  cat /sys/fs/cgroup/cpu.max 2>&1; echo "OMP=${OMP_NUM_THREADS:-unset}"; free -g; } > "$OUT/box.txt" 2>&1
if [ "${RUN_TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$OUT/gpu_tests.log" 2>&1 || { echo "gpu tests failed"; tail -40 "$OUT/gpu_tests.log"; exit 1; }
  tail -3 "$OUT/gpu_tests.log"
fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench1.json" 2> "$OUT/bench1.err" \
  || { echo "bench1 failed"; tail -20 "$OUT/bench1.err"; exit 1; }
cut -c1-400 "$OUT/bench1.json"
for c in ${CONFIGS:-2 3 4}; do
  timeout -k 10 240 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline \
    > "$OUT/bench$c.json" 2> "$OUT/bench$c.err" || { echo "bench$c failed"; tail -20 "$OUT/bench$c.err"; exit 1; }
  cut -c1-300 "$OUT/bench$c.json"
done
