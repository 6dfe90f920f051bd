#!/bin/bash
# PPO / env kernel tests on the current tree, then one cell (or a seed subset of one cell) of the
# pre-registered intermediate recipe (profiles/r5/reward/PREREGISTERED.md):
#   bash tools/r5/gpu_b2.sh COND HIDDEN "SEEDS" OUTNAME
set -o pipefail
mkdir -p gpurun_out/r5b
timeout -k 10 600 python -u -m pytest tests/test_ppo_fused_gpu.py tests/test_env_parity_gpu.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r5b/ppo_tests_$4.log 2>&1 || { tail -20 gpurun_out/r5b/ppo_tests_$4.log; exit 1; }
tail -1 gpurun_out/r5b/ppo_tests_$4.log
COND=$1 HID=$2 SEEDS="$3" E=256 T=128 M=512 EPISODES=24000 RUN_LIMIT=1000 \
  OUT=gpurun_out/r5_reward/$4 bash tools/reward_cell.sh
