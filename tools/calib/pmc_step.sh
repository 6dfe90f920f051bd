#!/bin/bash
# HBM traffic of hwy_step_kernel from PMC counters, calibrated (MI355X_MICROARCH.md: FETCH_SIZE /
# WRITE_SIZE in separate passes; non-16-B widths calibrated on a known byte count in the same
# access pattern).  Run on the GPU box from the repo root:  bash tools/calib/pmc_step.sh
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/calib/pmc_calib.hip \
  -o tools/calib/libpmc_calib.so
mkdir -p gpurun_out/pmc_step
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_step/fetch \
  -- python3 tools/calib/pmc_step.py > gpurun_out/pmc_step/fetch.log 2>&1
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_step/write \
  -- python3 tools/calib/pmc_step.py > gpurun_out/pmc_step/write.log 2>&1
python3 tools/calib/pmc_summarize.py gpurun_out/pmc_step
