#!/bin/bash
# Pricing of the 4,096-row minibatch step's fixed costs: per-kernel times of the product library,
# the dev build with Adam's tile writes skipped / Adam empty (HWY_PPO_SKIP=1 / 2, WRONG results,
# timing only), and the row kernel's per-phase clocks (prof build)
set -o pipefail
export PROBE_KT=1
H=highway-rope-ppo_amd/hwy
mkdir -p gpurun_out/ab3
for rep in 1 2; do
  for mb in 4096 16384; do
    timeout -k 10 120 python -u tools/probe_ppo_time.py 256 10 $mb 60 2>/dev/null | sed "s/^/product mb=$mb /" || exit 1
  done
  for sk in 0 1 2; do
    HWY_PPO_SKIP=$sk HWY_LIB=$H/libhwy_dev.so timeout -k 10 120 python -u tools/probe_ppo_time.py 256 10 4096 60 2>/dev/null \
      | sed "s/^/dev skip=$sk mb=4096 /" || exit 1
  done
done
timeout -k 10 120 python -u tools/probe_ppo_sections.py 256 4096 > gpurun_out/ab3/sections_4096.log 2>&1 || exit 1
cat gpurun_out/ab3/sections_4096.log
