#!/bin/bash
# Round-2 reward-recipe exploration on one MI355X: GPU tests, then lockstep training runs at
# E=4096 (sorted, h256, lr 3e-4, 8 epochs) for each "T:M" rollout/minibatch pair given.
set -u
OUT=${OUT:-gpurun_out/r2a}
mkdir -p "$OUT"
if [ "${RUN_TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > "$OUT/gpu_tests.log" 2>&1 || { echo "gpu tests failed"; tail -30 "$OUT/gpu_tests.log"; exit 1; }
  tail -3 "$OUT/gpu_tests.log"
fi
for tm in "$@"; do
  T=${tm%%:*}; M=${tm##*:}
  timeout -k 10 ${RUN_LIMIT:-420} python -u tools/train_parity.py --seeds ${SEEDS:-42} \
    --num-envs ${E:-4096} --rollout $T --minibatches $M --episodes ${EPISODES:-150000} \
    --eval-interval ${EVAL_INTERVAL:-2000} --lr ${LR:-3e-4} --out "$OUT/t${T}_m$M" \
    > "$OUT/t${T}_m$M.log" 2>&1 || { echo "train T=$T M=$M failed rc=$?"; tail -20 "$OUT/t${T}_m$M.log"; exit 1; }
  grep '"final_reward"\|mean_final' "$OUT/t${T}_m$M.log" | cut -c1-400
done
