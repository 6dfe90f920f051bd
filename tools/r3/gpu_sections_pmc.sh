#!/bin/bash
# Section clocks, then the configs[2]/[4] PMC passes (tools/r3/pmc_workload.sh).
set -o pipefail
bash tools/r3/sections.sh && \
CONFIG=2 bash tools/r3/pmc_workload.sh > gpurun_out/r3/pmc_c2.log 2>&1 && \
CONFIG=4 bash tools/r3/pmc_workload.sh > gpurun_out/r3/pmc_c4.log 2>&1
rc=$?
tail -4 gpurun_out/r3/pmc_c2.log gpurun_out/r3/pmc_c4.log 2>/dev/null
exit $rc
