#!/bin/bash
# The round's measurement record on one MI355X, run from the repo root on the GPU box; each step
# is time-limited and a failing step ends the script.  Everything lands in $OUT (default
# gpurun_out/measure); copy what is judged into profiles/<round>/measure/.
#   PART=tests  GPU test suite (TESTS="tests/x.py ..." limits it) + smoke + the default bench line
#   PART=lines  bench lines: configs[1] at T = 128, configs[2]-[4], configs[4]'s PE / hidden points
#   PART=prof   rocprofv3 --kernel-trace --stats of the configs[1] (T = 32 and 128) / configs[2]
#               benches -> kernel_stats_c<C>.txt (tools/summarize_stats.py)
#   PART=all    (default) the three in order
set -o pipefail
OUT=${OUT:-gpurun_out/measure}
mkdir -p "$OUT"
R=$(pwd)
step() { echo "[measure] $*"; }

tests() {
  step gpu tests
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 \
    --timeout-method thread > "$OUT/gpu_tests.log" 2>&1; local rc=$?
  tail -3 "$OUT/gpu_tests.log"
  [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" "$OUT/gpu_tests.log" | head -20; return $rc; }
  step smoke
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || return 1
  step bench default
  timeout -k 10 400 python -u bench.py > "$OUT/bench_c1.json" 2> "$OUT/bench_c1.err" || { tail -20 "$OUT/bench_c1.err"; return 1; }
  python3 - "$OUT/bench_c1.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print("value", d["value"], "ms/step", d["ms_per_step"], "mb_us", r["avg_launch_us"], "frac", r["frac"],
      "frac_req", r.get("frac_required"))
print("per_kernel", json.dumps(r.get("per_kernel")))
print("env", d["roofline_env_step"]["avg_launch_ms"], "breakdown", d.get("breakdown_ms"))
PY
}

lines() {
  local spec tag
  for spec in "1 --rollout 128" "2" "3" "4" "4 --pe rope --order shuffled --hidden 512" \
              "4 --pe rank --order shuffled --hidden 384" "4 --pe dist --order sorted"; do
    tag=$(echo "$spec" | tr -d ' -')
    step bench c$tag
    timeout -k 10 300 python bench.py --config $spec --steps 10 --warmup 3 --no-cpu-baseline \
      > "$OUT/bench_c$tag.json" 2> "$OUT/bench_c$tag.err" || { tail -20 "$OUT/bench_c$tag.err"; return 1; }
    cut -c1-160 "$OUT/bench_c$tag.json"
  done
}

prof() {
  local c S
  cd /tmp && export TMPDIR=/tmp && cd "$R"
  local spec
  for spec in "1" "2" "1 --rollout 128"; do
    c=$(echo "$spec" | tr -d ' -')
    step rocprof c$c
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c$c" -o run -- python3 bench.py \
      --config $spec --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/bench_prof_c$c.log" 2>&1 || { tail -20 "$OUT/bench_prof_c$c.log"; return 1; }
    S=$(ls "$OUT"/prof_c$c/run_kernel_stats.csv "$OUT"/prof_c$c/*/run_kernel_stats.csv \
          "$OUT"/prof_c$c/run_results.db "$OUT"/prof_c$c/*/run_results.db 2>/dev/null | head -1)
    python3 tools/summarize_stats.py "$S" 16 > "$OUT/kernel_stats_c$c.txt" && head -8 "$OUT/kernel_stats_c$c.txt"
    grep '^{' "$OUT/bench_prof_c$c.log" | tail -1 > "$OUT/bench_prof_c$c.json"
    rm -rf "$OUT/prof_c$c"  # the trace database (tens of MB); its summary is kept
  done
}

case ${PART:-all} in
  tests) tests ;;
  lines) lines ;;
  prof) prof ;;
  all) tests && lines && prof ;;
esac
rc=$?
step "done (rc $rc)"
exit $rc
