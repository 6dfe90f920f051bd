#!/bin/bash
# One reward-parity cell of the many-env recipe on one MI355X: E lockstep envs,
# T rollout steps, 32 minibatches, 8 epochs, lr 3e-4; COND / HID pick the reference cell
# (artifacts/combined_validated_data-final-run.csv); EPISODES budget (updates ~ the reference's
# ~125), evaluated 30 times per run; seeds 42, 1042, ..., 9042 (the first three are the
# reference's).  EXTRA passes further tools/train_parity.py options (--obs-vehicles 30 --order
# shuffled for the configs[2]/[4] workloads).  Writes OUT/summary.jsonl and OUT/stats.json.
set -u
COND=${COND:-sorted}; HID=${HID:-256}; E=${E:-4096}; T=${T:-128}; M=${M:-32}
EPISODES=${EPISODES:-320000}
OUT=${OUT:-gpurun_out/reward/${COND}_h${HID}_e${E}_t${T}}
EXTRA=${EXTRA:-}
SEEDS=${SEEDS:-42 1042 2042 3042 4042 5042 6042 7042 8042 9042}
mkdir -p "$OUT"
[ -n "${KEEP:-}" ] || rm -f "$OUT/summary.jsonl"
timeout -k 10 ${RUN_LIMIT:-1000} python -u tools/train_parity.py --seeds $SEEDS \
  --num-envs $E --rollout $T --minibatches $M --episodes $EPISODES --condition $COND \
  --hidden $HID --eval-interval $(( EPISODES / 30 )) --out "$OUT" $EXTRA >> "$OUT/train.log" 2>&1
rc=$?
find "$OUT" -name '*.pth' -delete
find "$OUT" -type d -name artifacts -prune -exec rm -rf {} +
[ -s "$OUT/summary.jsonl" ] && python tools/recipe_stats.py "$OUT" --note "$COND h$HID E=$E T=$T $EPISODES episodes $EXTRA" > "$OUT/stats.json"
grep -h '"mean\|matched' "$OUT/stats.json" 2>/dev/null | head -8
exit $rc
