#!/bin/bash
# PMC passes over the fused PPO kernels (development aid): pmc_ppo.sh <kernel regex> <tag>
set -e
R=$(pwd)
K=${1:-ppo_rows}
T=${2:-base}
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/pmcppo
i=0
for set in "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum" \
           "TCP_TCR_TCP_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum" \
           "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum" \
           "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $set --kernel-include-regex "$K" -d $R/gpurun_out/pmcppo/${T}_$i -o run --output-format csv -- python3 $R/tools/probe_ppo_time.py 256 2
done
