#!/bin/bash
# hwy_step timing: product vs variants at 4096 / 8192 / 16384 / 32768 envs (probe_step.py)
set -o pipefail
for rep in 1 2; do
  for lib in libhwy.so $(for v in $VARS; do echo libhwy_$v.so; done); do
    HWY_LIB=$PWD/highway-rope-ppo_amd/hwy/$lib timeout -k 10 90 python -u tools/probe_step.py 4096 8192 16384 32768 | sed "s/^/$lib /" || exit 1
  done
done
