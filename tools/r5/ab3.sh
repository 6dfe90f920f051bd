#!/bin/bash
# Pricing of the 4,096-row minibatch step's fixed costs: per-kernel times of the product library,
# the dev build with Adam's tile writes skipped / Adam empty (HWY_PPO_SKIP=1 / 2, WRONG results,
# timing only), and the row kernel's per-phase clocks (prof build)
set -o pipefail
export PROBE_KT=1
H=highway-rope-ppo_amd/hwy
mkdir -p gpurun_out/ab3
timeout -k 10 400 python -u -m pytest tests/test_env_parity_gpu.py tests/test_kernels_gpu.py tests/test_ppo_fused_gpu.py -x -q --timeout 200 \
  --timeout-method thread > gpurun_out/ab3/env_tests.log 2>&1 || { tail -20 gpurun_out/ab3/env_tests.log; exit 1; }
tail -1 gpurun_out/ab3/env_tests.log
for rep in 1 2; do
  for mb in 4096 16384; do
    timeout -k 10 120 python -u tools/probe_ppo_time.py 256 10 $mb 60 2>/dev/null | sed "s/^/product mb=$mb /" || exit 1
  done
  for kn in "HWY_ADAM_FLAT=1" "HWY_ADAM_FLAT=0" "HWY_PPO_SKIP=1" "HWY_PPO_SKIP=2"; do
    env $kn HWY_LIB=$H/libhwy_dev.so timeout -k 10 120 python -u tools/probe_ppo_time.py 256 10 4096 60 2>/dev/null \
      | sed "s/^/dev $kn mb=4096 /" || exit 1
  done
done
timeout -k 10 120 python -u tools/probe_ppo_sections.py 256 4096 > gpurun_out/ab3/sections_4096.log 2>&1 || exit 1
cat gpurun_out/ab3/sections_4096.log
# hwy_step instruction pricing of the current tree: MOBIL (skip1), collisions (skip4), obs rank (skip64)
VARS="skip1 skip4 skip64" MODE=pmc REPS=1 bash tools/ab.sh 2>&1 | grep launches &&
VARS="" MODE=step REPS=3 ENVS="4096 16384" bash tools/ab.sh 2>&1 | grep env-steps
# kernel-trace durations of the 4,096-row step (to set beside the per-kernel graph times above)
VARS="" MODE=kt MB=4096 REPS=1 bash tools/ab.sh 2>&1 | tail -8
