#!/bin/bash
# GPU test suite + smoke + default bench on the box (each step time-limited, chained with &&).
# OUT=gpurun_out/<dir>; TESTS="tests/x.py ..." limits the suite.
set -o pipefail
OUT=${OUT:-gpurun_out/r5}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread \
  > "$OUT/gpu_tests.log" 2>&1; rc=$?
tail -3 "$OUT/gpu_tests.log"
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" "$OUT/gpu_tests.log" | head -20; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 && \
timeout -k 10 400 python -u bench.py > "$OUT/bench_c1.json" 2> "$OUT/bench_c1.err" && \
cut -c1-300 "$OUT/bench_c1.json" && python3 - "$OUT/bench_c1.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print("value", d["value"], "ms/step", d["ms_per_step"], "mb_us", r["avg_launch_us"], "frac", r["frac"],
      "frac_req", r.get("frac_required"))
print("per_kernel", json.dumps(r.get("per_kernel")))
print("env", d["roofline_env_step"]["avg_launch_ms"], "breakdown", d.get("breakdown_ms"))
PY
