#!/bin/bash
# Reward parity of the lockstep (vectorised) loop: $CONDITION (default sorted) / h256 / bs64 /
# 1500 episodes at seeds 42 1042 2042 (or $SEEDS), one process per seed, for each E given
# (default 16 64).
set -u
OUT=${OUT:-gpurun_out/train_vec}
mkdir -p "$OUT"
Es=("$@")
[ ${#Es[@]} -eq 0 ] && Es=(16 64)
for E in "${Es[@]}"; do
  pids=()
  for s in ${SEEDS:-42 1042 2042}; do
    timeout -k 10 900 python -u tools/train_parity.py --seeds $s --num-envs $E \
      --condition ${CONDITION:-sorted} --out "$OUT/e$E" > "$OUT/e${E}_seed$s.log" 2>&1 &
    pids+=($!)
  done
  for p in "${pids[@]}"; do wait $p || exit $?; done
done
