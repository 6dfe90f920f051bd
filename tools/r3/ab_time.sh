#!/bin/bash
# minibatch-step times of the product library against variants (libhwy_<V>.so, V in $VARS),
# interleaved; SHAPES="H:rows:S ..." (default the configs[1] and configs[4] h256 / h384 steps)
set -o pipefail
for shp in ${SHAPES:-256:16384:60 256:32768:120 384:32768:120}; do
  IFS=: read H mb S <<< "$shp"
  for rep in 1 2; do
    for lib in libhwy.so $(for v in $VARS; do echo libhwy_$v.so; done); do
      HWY_LIB=$PWD/highway-rope-ppo_amd/hwy/$lib timeout -k 10 60 python -u tools/probe_ppo_time.py $H 6 $mb $S | sed "s/^/$lib mb=$mb S=$S /" || exit 1
    done
  done
done
