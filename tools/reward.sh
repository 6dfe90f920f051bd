#!/bin/bash
# Reward-parity recipes on one MI355X, run from the repo root on the GPU box.
# Every part first runs the PPO / env kernel parity tests on the tree it trains with.
#   PART=A  the bench line's recipe: configs[1] at T = 32 (E 4,096, 32 minibatches, 80,000
#           episodes), sorted h256, seeds 42, 1042, ..., 9042
#   PART=B  the pre-registered intermediate recipe (profiles/r5/reward/PREREGISTERED.md: E 256,
#           T 128, 512 minibatches of 64, 24,000 episodes) for the reference's six cells;
#           CELLS="cond:hidden ..." limits it, SEEDS="..." runs a subset of one cell's seeds into
#           <cell>_<TAG> (merge the halves with tools/recipe_stats.py)
# Any other recipe is one tools/reward_cell.sh call (COND HID E T M EPISODES EXTRA env vars).
set -o pipefail
OUT=${OUT:-gpurun_out/reward}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_ppo_fused_gpu.py tests/test_env_parity_gpu.py \
  tests/test_kernels_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/kernel_tests${TAG:+_$TAG}.log" 2>&1 || { tail -20 "$OUT/kernel_tests${TAG:+_$TAG}.log"; exit 1; }
tail -1 "$OUT/kernel_tests${TAG:+_$TAG}.log"
case ${PART:-A} in
A)
  COND=sorted HID=256 E=4096 T=32 M=32 EPISODES=80000 RUN_LIMIT=400 \
    OUT=$OUT/sorted_h256_e4096_t32 bash tools/reward_cell.sh ;;
B)
  for cell in ${CELLS:-sorted:256 sorted:384 sorted:512 shuffled_rope:256 shuffled_distpe:256 shuffled_rankpe:256}; do
    c=${cell%%:*}; h=${cell##*:}
    echo "[reward B] $c h$h"
    COND=$c HID=$h E=256 T=128 M=512 EPISODES=24000 RUN_LIMIT=1000 \
      OUT=$OUT/${c}_h${h}_e256_t128${TAG:+_$TAG} bash tools/reward_cell.sh || exit 1
  done ;;
esac
