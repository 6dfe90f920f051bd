#!/bin/bash
# ppo_rows_k (libhwy.so) against ppo_rows_c64 (libhwy_c64.so): the fused-step tests on the product
# library, interleaved minibatch-step times, a kernel trace of each.
set -o pipefail
R=$(pwd); O=$R/gpurun_out/rk; mkdir -p $O; H=$R/highway-rope-ppo_amd/hwy
timeout -k 10 900 python -u -m pytest tests/test_ppo_fused_gpu.py -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; grep -E "FAIL|ERROR" $O/tests.log | head -20; tail -2 $O/tests.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for shp in 256:16384:60 256:32768:120 256:32768:240; do
  IFS=: read Hd mb S <<< "$shp"
  for rep in 1 2; do
    for lib in libhwy.so libhwy_c64.so; do
      HWY_LIB=$H/$lib HWY_SPLIT_STEP=1 timeout -k 10 90 python -u tools/probe_ppo_time.py $Hd 10 $mb $S \
        | sed "s/^/$lib H=$Hd mb=$mb S=$S /" | grep -v sha1 || exit 1
    done
  done
done
cd /tmp && export TMPDIR=/tmp
for lib in libhwy.so libhwy_c64.so; do
  HWY_LIB=$H/$lib timeout -s KILL 120 rocprofv3 --kernel-trace --stats --kernel-include-regex ppo_ \
    -d $O/kt_${lib%.so} -o run --output-format csv -- python3 $R/tools/probe_ppo_time.py 256 3 16384 > $O/kt_${lib%.so}.log 2>&1 || { echo "kt $lib failed"; tail -3 $O/kt_${lib%.so}.log; exit 1; }
  echo "== $lib"; python3 $R/tools/summarize_stats.py "$(find $O/kt_${lib%.so} -name '*kernel_stats.csv' | head -1)" 4
done
