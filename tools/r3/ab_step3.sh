#!/bin/bash
# hwy_step timing, product vs variants ($VARS): configs[1] shapes (probe_step.py) and the
# 30-row shuffled PE shapes (probe_step_pe.py)
set -o pipefail
for rep in 1 2; do
  for lib in libhwy.so $(for v in $VARS; do echo libhwy_$v.so; done); do
    export HWY_LIB=$PWD/highway-rope-ppo_amd/hwy/$lib
    timeout -k 10 90 python -u tools/probe_step.py 4096 32768 | sed "s/^/$lib /" || exit 1
    for pe in ${PES:-rope rank}; do
      timeout -k 10 90 python -u tools/r3/probe_step_pe.py $pe 16384 | sed "s/^/$lib /" || exit 1
    done
  done
done
