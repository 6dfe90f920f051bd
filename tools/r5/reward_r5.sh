#!/bin/bash
# Round-5 reward evidence (profiles/r5/reward/PREREGISTERED.md), one MI355X, run from the repo root.
#   PART=A: the bench line's recipe (E 4,096, T 32, 32 minibatches, 80,000 episodes), sorted h256
#   PART=B: the intermediate recipe (E 256, T 128, 512 minibatches of 64, 24,000 episodes) for the
#           six reference cells; CELLS limits it ("cond:hidden ...")
set -o pipefail
OUT=${OUT:-gpurun_out/r5_reward}
mkdir -p "$OUT"
case ${PART:-A} in
A)
  COND=sorted HID=256 E=4096 T=32 M=32 EPISODES=80000 RUN_LIMIT=400 \
    OUT=$OUT/sorted_h256_e4096_t32 bash tools/reward_cell.sh ;;
B)
  for cell in ${CELLS:-sorted:256 sorted:384 sorted:512 shuffled_rope:256 shuffled_distpe:256 shuffled_rankpe:256}; do
    c=${cell%%:*}; h=${cell##*:}
    echo "[reward B] $c h$h"
    COND=$c HID=$h E=256 T=128 M=512 EPISODES=24000 RUN_LIMIT=900 \
      OUT=$OUT/${c}_h${h}_e256_t128 bash tools/reward_cell.sh || exit 1
  done ;;
esac
