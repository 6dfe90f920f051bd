#!/bin/bash
# Effective clock and MFMA busy of ppo_rows* / ppo_wgrad for the product library and a variant
# (GRBM_GUI_ACTIVE / 8 / wall = clock; SQ_VALU_MFMA_BUSY_CYCLES / GRBM_GUI_ACTIVE / 32 CUs per XCD)
R=$(pwd)
V=${V:-nocmp}
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/pmcclk
for lib in libhwy.so libhwy_$V.so; do
  export HWY_LIB=$R/highway-rope-ppo_amd/hwy/$lib
  timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES \
    --kernel-include-regex "ppo_(rows|wgrad)" -d $R/gpurun_out/pmcclk/$lib -o run --output-format csv \
    -- python3 $R/tools/probe_ppo_time.py 256 2 16384 > $R/gpurun_out/pmcclk/$lib.log 2>&1 || { echo "pmc $lib failed"; tail -5 $R/gpurun_out/pmcclk/$lib.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats --kernel-include-regex "ppo_" \
    -d $R/gpurun_out/pmcclk/kt_$lib -o run --output-format csv \
    -- python3 $R/tools/probe_ppo_time.py 256 2 16384 > $R/gpurun_out/pmcclk/kt_$lib.log 2>&1 || { echo "kt $lib failed"; exit 1; }
done
echo pmc ok
