#!/bin/bash
# 2-rank gloo rehearsal of bench.py's N > 1 path on one GPU: the full JSON line, for the
# all-reduce-share cross-check
set -o pipefail
OUT=${OUT:-gpurun_out/r6diag}
mkdir -p "$OUT"
export HWY_BENCH_DIST_BACKEND=gloo
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 \
  --envs 256 --rollout 8 --minibatches 4 --epochs 2 > "$OUT/dist2.json" 2> "$OUT/dist2.err" || { tail -30 "$OUT/dist2.err"; exit 1; }
python3 - "$OUT/dist2.json" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d["roofline"]
print("ms_per_step", d["ms_per_step"], "breakdown", d["breakdown_ms"])
print("avg_launch_us", r["avg_launch_us"], "update_host_us_per_step", r["update_host_us_per_step"],
      "share", r["allreduce_share_of_step"], "mode", d["config"]["epoch_graph_collectives"])
print("allreduce", r["allreduce"])
PY
