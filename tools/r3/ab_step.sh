#!/bin/bash
# env-step parity tests on the product library, then hwy_step timing: product vs variant(s)
set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 600 python -u -m pytest tests/test_env_parity_gpu.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r3/ab_step_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r3/ab_step_tests.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for lib in libhwy.so $(for v in $VARS; do echo libhwy_$v.so; done); do
    HWY_LIB=$PWD/highway-rope-ppo_amd/hwy/$lib timeout -k 10 60 python -u tools/probe_step.py 4096 16384 | sed "s/^/$lib /" || exit 1
  done
done
