#!/bin/bash
# PPO kernel tests on the current tree, then cells 1-2 of the pre-registered intermediate recipe
set -o pipefail
mkdir -p gpurun_out/r5b
timeout -k 10 600 python -u -m pytest tests/test_ppo_fused_gpu.py tests/test_env_parity_gpu.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r5b/ppo_tests.log 2>&1 || { tail -20 gpurun_out/r5b/ppo_tests.log; exit 1; }
tail -1 gpurun_out/r5b/ppo_tests.log
PART=B CELLS="${CELLS:-sorted:256 sorted:384}" bash tools/r5/reward_r5.sh
