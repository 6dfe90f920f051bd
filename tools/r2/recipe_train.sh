#!/bin/bash
# The many-env reward recipe on one MI355X: E lockstep envs, T rollout steps,
# M minibatches, 8 epochs, lr 3e-4, h256, sorted; EPISODES budget, evaluated 30 times per run
# like the reference (1500 episodes / every 50); one process, seeds in turn.
set -u
OUT=${OUT:-gpurun_out/r2_recipe}
E=${E:-4096}; T=${T:-32}; M=${M:-32}; EPISODES=${EPISODES:-80000}
COND=${COND:-sorted}
mkdir -p "$OUT"
timeout -k 10 ${RUN_LIMIT:-900} python -u tools/train_parity.py --seeds ${SEEDS:-42 1042 2042} \
  --num-envs $E --rollout $T --minibatches $M --episodes $EPISODES --condition $COND \
  --eval-interval $(( EPISODES / 30 )) --out "$OUT" > "$OUT/train.log" 2>&1
rc=$?
find "$OUT" -name '*.pth' -delete
find "$OUT" -type d -name artifacts -prune -exec rm -rf {} +  # per-episode JSON / plots: large
grep '"final_reward"\|mean_final' "$OUT/train.log" | cut -c1-300
exit $rc
