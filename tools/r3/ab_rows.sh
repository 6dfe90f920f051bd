#!/bin/bash
# ppo_rows A/B: the fused-gradient parity tests on the product library, then the minibatch-step
# time of the product library against a variant (HWY_LIB), both at 16,384 and 32,768 rows.
set -o pipefail
mkdir -p gpurun_out/r3
V=${V:-nocmp}
timeout -k 10 600 python -u -m pytest tests/test_ppo_fused_gpu.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r3/ab_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r3/ab_tests.log
[ $rc -eq 0 ] || exit $rc
for mb in 16384 32768; do
  for lib in libhwy.so libhwy_$V.so libhwy.so libhwy_$V.so; do
    HWY_LIB=$PWD/highway-rope-ppo_amd/hwy/$lib timeout -k 10 60 python -u tools/probe_ppo_time.py 256 10 $mb | sed "s/^/$lib mb=$mb /" || exit 1
  done
done
