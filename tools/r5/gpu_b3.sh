#!/bin/bash
# sorted h512 seeds 5042-9042 of the pre-registered intermediate recipe, then the env kernel's
# section clocks at 4,096 envs (prof build)
set -o pipefail
SEEDS="5042 6042 7042 8042 9042" PART=B CELLS="sorted:512" TAG=b OUT=gpurun_out/r5_reward \
  bash tools/reward.sh || exit 1
timeout -k 10 120 python -u tools/probe_sections.py 4096 > gpurun_out/r5_reward/env_sections.log 2>&1 || exit 1
cat gpurun_out/r5_reward/env_sections.log
