#!/bin/bash
# Round-5 first GPU session: the 16-row weight-stream micro-benchmark, kernel stats of the T = 32
# bench line, and ppo_rows section clocks at 4,096 rows (16-row tiles) and 16,384 (64-row tiles).
set -o pipefail
OUT=${OUT:-gpurun_out/r5p1}
mkdir -p "$OUT"
R=$(pwd)
echo "[p1] micro"
timeout -k 10 120 tools/micro/rows16_stream > "$OUT/rows16_stream.log" 2>&1 || { tail -5 "$OUT/rows16_stream.log"; exit 1; }
cat "$OUT/rows16_stream.log"
echo "[p1] sections 4096"
timeout -k 10 120 python3 -u tools/probe_ppo_sections.py 256 4096 > "$OUT/sections_4096.log" 2>&1 || { tail -5 "$OUT/sections_4096.log"; exit 1; }
cat "$OUT/sections_4096.log"
echo "[p1] bench t32 under rocprof"
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_t32" -o run -- python3 bench.py --rollout 32 --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/bench_prof_t32.log" 2>&1 || { tail -20 "$OUT/bench_prof_t32.log"; exit 1; }
S=$(ls "$OUT"/prof_t32/run_kernel_stats.csv "$OUT"/prof_t32/*/run_kernel_stats.csv 2>/dev/null | head -1)
python3 tools/summarize_stats.py "$S" 12 > "$OUT/kernel_stats_t32.txt" && cat "$OUT/kernel_stats_t32.txt"
echo "[p1] done"
