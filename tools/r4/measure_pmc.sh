#!/bin/bash
# Round-4 measurement set, part 2: PMC of hwy_step (instruction counts, calibrated HBM bytes) at
# configs[1], the minibatch-step HBM-side traffic at 16,384 rows (configs[1]), and both at the
# configs[2] / configs[4] workloads (tools/r3/pmc_workload.sh).  The JSON summaries the tools
# write under profiles/ are copied to $OUT/pmc_json.
set -u
OUT=${OUT:-gpurun_out/r4m}
mkdir -p "$OUT"
R=$(pwd)
step() { echo "[measure] $*"; }
step pmc hwy_step instruction counts
bash tools/pmc_kernel.sh hwy_step step python3 $R/tools/probe_step.py 4096 > "$OUT/pmc_step_insts.log" 2>&1 || { tail -20 "$OUT/pmc_step_insts.log"; exit 1; }
python3 tools/calib/valu_summarize.py gpurun_out/pmck > /dev/null || exit 1
step pmc hwy_step bytes
bash tools/calib/pmc_step.sh > "$OUT/pmc_step_bytes.log" 2>&1 || { tail -20 "$OUT/pmc_step_bytes.log"; exit 1; }
step pmc ppo 16384
MB=16384 bash tools/pmc_ppo_traffic.sh > "$OUT/pmc_ppo_16384.log" 2>&1 || { tail -20 "$OUT/pmc_ppo_16384.log"; exit 1; }
grep -E "hbm_side_bytes_per_step" "$OUT/pmc_ppo_16384.log"
for c in 2 4; do
  step pmc workload c$c
  CONFIG=$c bash tools/r3/pmc_workload.sh > "$OUT/pmc_c$c.log" 2>&1 || { tail -20 "$OUT/pmc_c$c.log"; exit 1; }
done
mkdir -p "$OUT/pmc_json" && cp profiles/hwy_step_*.json profiles/ppo_step_pmc*.json "$OUT/pmc_json/"
step done
