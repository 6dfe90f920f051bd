#!/bin/bash
# PMC passes (one rocprofv3 run per counter set) over one kernel (development aid):
#   pmc_kernel.sh <kernel regex> <tag> [command ...]   (default command: probe_ppo_time.py 256 2)
R=$(pwd)
K=${1:-ppo_wgrad}
T=${2:-base}
shift 2
CMD=("$@")
[ ${#CMD[@]} -eq 0 ] && CMD=(python3 $R/tools/probe_ppo_time.py 256 2)
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/pmck
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVES" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-include-regex "$K" -d $R/gpurun_out/pmck/${T}_$i -o run \
    --output-format csv -- "${CMD[@]}" > $R/gpurun_out/pmck/${T}_$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/gpurun_out/pmck/${T}_$i.log; exit 1; }
done
python3 $R/tools/pmc_table.py $R/gpurun_out/pmck
