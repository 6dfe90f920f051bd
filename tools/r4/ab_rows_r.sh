#!/bin/bash
# ppo_rows_r (activations in registers) against ppo_rows_c64 (libhwy_c64.so): gradient tests of the
# fused step on the product library, then interleaved minibatch-step times (split = the two-call
# step) and a kernel trace of each library.
set -o pipefail
R=$(pwd); O=$R/gpurun_out/rr; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_ppo_fused_gpu.py -v --timeout 300 --timeout-method thread \
  -k "gradient_matches_autograd or single_call or matches_torch_update or golden or every_step" > $O/tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR" $O/tests.log | grep -E "FAIL|ERROR" | head -20; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
H=$R/highway-rope-ppo_amd/hwy
for shp in 256:16384:60 256:32768:120 256:32768:240; do
  IFS=: read Hd mb S <<< "$shp"
  for rep in 1 2; do
    for lib in libhwy.so libhwy_c64.so; do
      for sp in 0 1; do
        HWY_LIB=$H/$lib HWY_SPLIT_STEP=$sp timeout -k 10 90 python -u tools/probe_ppo_time.py $Hd 10 $mb $S \
          | sed "s/^/$lib split=$sp H=$Hd mb=$mb S=$S /" || exit 1
      done
    done
  done
done
cd /tmp && export TMPDIR=/tmp
for lib in libhwy.so libhwy_c64.so; do
  HWY_LIB=$H/$lib timeout -s KILL 120 rocprofv3 --kernel-trace --stats --kernel-include-regex ppo_ \
    -d $O/kt_${lib%.so} -o run --output-format csv -- python3 $R/tools/probe_ppo_time.py 256 3 16384 > $O/kt_${lib%.so}.log 2>&1 || { echo "kt $lib failed"; tail -3 $O/kt_${lib%.so}.log; exit 1; }
  echo "== $lib"; python3 $R/tools/summarize_stats.py "$(find $O/kt_${lib%.so} -name '*kernel_stats.csv' | head -1)" 8
done
