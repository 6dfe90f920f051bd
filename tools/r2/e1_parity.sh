# E = 1 reward parity (the reference's own loop through ExperimentRunner) for the north-star
# cell, seeds 42 / 1042 / 2042 in three processes, with the current kernels
OUT=${OUT:-gpurun_out/train_e1_r2}
mkdir -p $OUT
( while true; do sleep 60; echo "[tick] $(date +%T) $(cat $OUT/*.log 2>/dev/null | grep -c Evaluating) evals"; done ) &
TICK=$!
pids=""
for s in ${SEEDS:-42 1042 2042}; do
  timeout -k 10 1000 python -u tools/train_parity.py --seeds $s --out $OUT/seed$s > $OUT/seed$s.log 2>&1 &
  pids="$pids $!"
done
rc=0
for p in $pids; do wait $p || rc=1; done
kill $TICK
cat $OUT/seed*/summary.jsonl
exit $rc
