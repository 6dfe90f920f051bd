#!/bin/bash
# Round-3 reward evidence on current kernels, E = 4096 lockstep envs, 10 seeds each:
# the north-star cell at both benched recipes (T 128 / 320k episodes, T 32 / 80k episodes) and the
# three PE conditions of configs[2]/[4] at h256 (T 128).  Run from the repo root on the GPU box.
set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 60 python -u tools/probe_ppo_time.py 256 5 16384 > gpurun_out/r3/ppo_time.log 2>&1 && \
cat gpurun_out/r3/ppo_time.log && \
COND=sorted HID=256 T=128 EPISODES=320000 RUN_LIMIT=400 OUT=gpurun_out/r3_reward/sorted_h256_e4096_t128 bash tools/reward_cell.sh && \
COND=sorted HID=256 T=32 EPISODES=80000 RUN_LIMIT=300 OUT=gpurun_out/r3_reward/sorted_h256_e4096_t32 bash tools/reward_cell.sh && \
for c in ${CELLS:-shuffled_rope shuffled_distpe shuffled_rankpe}; do
  COND=$c HID=256 T=128 EPISODES=320000 RUN_LIMIT=400 OUT=gpurun_out/r3_reward/${c}_h256_e4096_t128 bash tools/reward_cell.sh || exit 1
done
