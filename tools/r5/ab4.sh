#!/bin/bash
# hwy_step after the wave-mask rework: parity tests, VALU / SALU per launch, step time, section clocks
set -o pipefail
mkdir -p gpurun_out/ab4
timeout -k 10 400 python -u -m pytest tests/test_env_parity_gpu.py tests/test_kernels_gpu.py -x -q --timeout 200 \
  --timeout-method thread > gpurun_out/ab4/env_tests.log 2>&1 || { tail -20 gpurun_out/ab4/env_tests.log; exit 1; }
tail -1 gpurun_out/ab4/env_tests.log
VARS="" MODE=pmc REPS=1 bash tools/ab.sh 2>&1 | grep launches &&
VARS="" MODE=step REPS=3 ENVS="4096 16384" bash tools/ab.sh 2>&1 | grep env-steps &&
timeout -k 10 120 python -u tools/probe_sections.py 4096 > gpurun_out/ab4/env_sections.log 2>&1 &&
cat gpurun_out/ab4/env_sections.log
