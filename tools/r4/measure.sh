#!/bin/bash
# Round-4 measurement set, part 1 (one MI355X): bench lines for configs 1-4 (+ configs[4]'s PE /
# hidden points and the T = 32 recipe), rocprofv3 kernel stats of the configs[1] and configs[2]
# benches.  Everything lands in $OUT; copy what is judged into profiles/r4/.
set -u
OUT=${OUT:-gpurun_out/r4m}
mkdir -p "$OUT"
R=$(pwd)
step() { echo "[measure] $*"; }
step bench c1
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > "$OUT/bench_c1.json" 2> "$OUT/bench_c1.err" || { tail -20 "$OUT/bench_c1.err"; exit 1; }
cut -c1-200 "$OUT/bench_c1.json"
for spec in "1 --rollout 32" "2" "3" "4" "4 --pe rope --order shuffled --hidden 512" "4 --pe rank --order shuffled --hidden 384" "4 --pe dist --order sorted"; do
  tag=$(echo "$spec" | tr -d ' -' )
  step bench c$tag
  timeout -k 10 300 python bench.py --config $spec --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/bench_c$tag.json" 2> "$OUT/bench_c$tag.err" || { tail -20 "$OUT/bench_c$tag.err"; exit 1; }
  cut -c1-160 "$OUT/bench_c$tag.json"
done
cd /tmp && export TMPDIR=/tmp && cd "$R"
for c in 1 2; do
  step rocprof c$c
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c$c" -o run -- python3 bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/bench_prof_c$c.log" 2>&1 || { tail -20 "$OUT/bench_prof_c$c.log"; exit 1; }
  S=$(ls "$OUT"/prof_c$c/run_kernel_stats.csv "$OUT"/prof_c$c/*/run_kernel_stats.csv "$OUT"/prof_c$c/run_results.db "$OUT"/prof_c$c/*/run_results.db 2>/dev/null | head -1)
  python3 tools/summarize_stats.py "$S" 16 > "$OUT/kernel_stats_c$c.txt" && head -8 "$OUT/kernel_stats_c$c.txt"
done
step done
