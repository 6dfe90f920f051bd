#!/bin/bash
# PMC passes of the round's measurement record (one MI355X, repo root, separate rocprofv3 passes
# per MI355X_MICROARCH.md): hwy_step instruction counts and calibrated HBM bytes at configs[1]
# (tools/pmc_kernel.sh, tools/calib/pmc_step.sh), the minibatch-step traffic of configs[1]'s
# 4,096-row step and the 16,384-row step (tools/pmc_ppo_traffic.sh), and both at the configs[2] /
# configs[4] workloads (tools/pmc_workload.sh).  The JSON summaries the tools write under
# profiles/ are copied to $OUT/pmc_json (gpurun merges back only gpurun_out/).
set -u
OUT=${OUT:-gpurun_out/measure}
mkdir -p "$OUT"
R=$(pwd)
step() { echo "[measure_pmc] $*"; }
step pmc hwy_step instruction counts
bash tools/pmc_kernel.sh hwy_step step python3 $R/tools/probe_step.py 4096 > "$OUT/pmc_step_insts.log" 2>&1 || { tail -20 "$OUT/pmc_step_insts.log"; exit 1; }
python3 tools/calib/valu_summarize.py gpurun_out/pmck > /dev/null || exit 1
step pmc hwy_step bytes
bash tools/calib/pmc_step.sh > "$OUT/pmc_step_bytes.log" 2>&1 || { tail -20 "$OUT/pmc_step_bytes.log"; exit 1; }
for mb in 4096 16384; do
  step pmc ppo $mb
  MB=$mb bash tools/pmc_ppo_traffic.sh > "$OUT/pmc_ppo_$mb.log" 2>&1 || { tail -20 "$OUT/pmc_ppo_$mb.log"; exit 1; }
  grep -E "hbm_side_bytes_per_step" "$OUT/pmc_ppo_$mb.log"
done
for c in ${CONFIGS:-2 4}; do
  step pmc workload c$c
  CONFIG=$c bash tools/pmc_workload.sh > "$OUT/pmc_c$c.log" 2>&1 || { tail -20 "$OUT/pmc_c$c.log"; exit 1; }
done
mkdir -p "$OUT/pmc_json" && cp profiles/hwy_step_*.json profiles/ppo_step_pmc*.json "$OUT/pmc_json/"
step done
