#!/bin/bash
# One parametrised A/B driver for kernel variants (replaces the round-2/3 one-off scripts).
# Variants are development builds `make -C highway-rope-ppo_amd/csrc variant V=<name> VEXTRA=...`
# -> hwy/libhwy_<name>.so; the product library libhwy.so is always the A side.  Run on the GPU box
# from the repo root:
#   MODE=ppo   VARS="v1 v2" [TESTS=1] [SHAPES="H:rows:S ..."] [REPS=2] bash tools/ab.sh
#              minibatch-step time (tools/probe_ppo_time.py), interleaved per shape
#   MODE=step  VARS=... [TESTS=1] [ENVS="4096 16384"] [REPS=3]   hwy_step time (tools/probe_step.py)
#   MODE=kt    VARS=... [WHAT=ppo|step] [MB=16384]   rocprofv3 kernel-trace averages per library
#   MODE=pmc   VARS=... [COUNTERS="SQ_INSTS_VALU ..."]  SQ instruction counts per hwy_step launch
#   MODE=act   VARS=... [ROWS="4096 16384 32768"]    ppo_act kernel-trace time (tools/probe_act.py)
# TESTS=1 first runs the parity tests of the touched kernel on the product library and every
# variant (tests/test_ppo_fused_gpu.py for ppo/act, tests/test_env_parity_gpu.py for step/pmc).
# KNOBS="NAME=v ..." (MODE=ppo): also runs the dev build (VARS must hold its name, e.g. dev) once
# per runtime knob setting (HWY_ADAM_FLAT=1, HWY_PPO_SKIP=1|2: timing-only pricing builds).
# PROBE_KT=1 prints each kernel's time too (hwy_ppo_time_kernels).
set -o pipefail
R=$(pwd)
H=$R/highway-rope-ppo_amd/hwy
OUT=$R/gpurun_out/ab_${MODE:-ppo}
mkdir -p "$OUT"
LIBS="libhwy.so $(for v in ${VARS:-}; do echo libhwy_$v.so; done)"
REPS=${REPS:-2}

run_tests() {  # test file
  for lib in $LIBS; do
    HWY_LIB=$H/$lib timeout -k 10 900 python -u -m pytest "$1" -x -q --timeout 300 \
      --timeout-method thread > "$OUT/tests_${lib%.so}.log" 2>&1 || {
        echo "tests failed on $lib"; tail -5 "$OUT/tests_${lib%.so}.log"; exit 1; }
    echo "$lib: $(tail -1 "$OUT/tests_${lib%.so}.log")"
  done
}

case ${MODE:-ppo} in
ppo)
  [ -n "${TESTS:-}" ] && run_tests tests/test_ppo_fused_gpu.py
  for shp in ${SHAPES:-256:16384:60 256:32768:120}; do
    IFS=: read Hd mb S <<< "$shp"
    for rep in $(seq $REPS); do
      for lib in $LIBS; do
        HWY_LIB=$H/$lib timeout -k 10 90 python -u tools/probe_ppo_time.py $Hd 10 $mb $S \
          | sed "s/^/$lib H=$Hd mb=$mb S=$S /" || exit 1
      done
      for kn in ${KNOBS:-}; do
        env $kn HWY_LIB=$H/libhwy_${VARS%% *}.so timeout -k 10 90 python -u tools/probe_ppo_time.py \
          $Hd 10 $mb $S | sed "s/^/${VARS%% *} $kn H=$Hd mb=$mb S=$S /" || exit 1
      done
    done
  done ;;
step)
  [ -n "${TESTS:-}" ] && run_tests tests/test_env_parity_gpu.py
  for rep in $(seq ${REPS:-3}); do
    for lib in $LIBS; do
      HWY_LIB=$H/$lib timeout -k 10 90 python -u tools/probe_step.py ${ENVS:-4096 16384} \
        | sed "s/^/$lib /" || exit 1
    done
  done ;;
kt|pmc|act)
  cd /tmp && export TMPDIR=/tmp
  for rep in $(seq $REPS); do
    for lib in $LIBS; do
      d=$OUT/${lib%.so}_$rep
      case $MODE in
        kt) if [ "${WHAT:-ppo}" = step ]; then prog="$R/tools/probe_step.py 4096"; rx=hwy_step
            else prog="$R/tools/probe_ppo_time.py 256 3 ${MB:-16384}"; rx=ppo_; fi
            prof="--kernel-trace --stats" ;;
        act) prog="$R/tools/probe_act.py ${ROWS:-4096 16384 32768}"; rx=ppo_act
             prof="--kernel-trace --stats" ;;
        pmc) prog="$R/tools/probe_step.py 4096"; rx=hwy_step
             prof="--pmc ${COUNTERS:-SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_WAVES}" ;;
      esac
      HWY_LIB=$H/$lib timeout -s KILL 120 rocprofv3 $prof --kernel-include-regex "$rx" \
        -d "$d" -o run --output-format csv -- python3 $prog > "$d.log" 2>&1 || {
          echo "$MODE $lib failed"; tail -3 "$d.log"; exit 1; }
      if [ $MODE = pmc ]; then
        python3 $R/tools/valu_summarize_ab.py "$(find "$d" -name '*counter_collection.csv' | head -1)" "$lib"
      else
        echo "== $lib rep $rep"
        python3 $R/tools/summarize_stats.py "$(find "$d" -name '*kernel_stats.csv' | head -1)" 6
      fi
    done
  done ;;
*) echo "unknown MODE=$MODE"; exit 2 ;;
esac
