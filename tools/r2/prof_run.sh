#!/bin/bash
# rocprofv3 kernel stats of the configs[1] bench + the PPO section clocks (prof build).
set -u
OUT=${OUT:-gpurun_out/r2p}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/bench_prof.log" 2>&1 || { echo "rocprof bench failed"; tail -20 "$OUT/bench_prof.log"; exit 1; }
grep '^{' "$OUT/bench_prof.log" | cut -c1-200
S=$(ls "$OUT"/prof/run_kernel_stats.csv "$OUT"/prof/*/run_kernel_stats.csv "$OUT"/prof/run_results.db "$OUT"/prof/*/run_results.db 2>/dev/null | head -1)
python3 tools/summarize_stats.py "$S" 16 > "$OUT/kernel_stats_top.txt" && cat "$OUT/kernel_stats_top.txt"
if [ "${SECTIONS:-1}" = 1 ]; then
  timeout -k 10 120 python3 tools/probe_ppo_sections.py 256 > "$OUT/sections.txt" 2>&1; cat "$OUT/sections.txt"
fi
