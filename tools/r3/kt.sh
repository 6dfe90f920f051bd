#!/bin/bash
# kernel-trace stats of the PPO minibatch step (probe_ppo_time) for the product library and variants
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/kt
for lib in libhwy.so $(for v in $VARS; do echo libhwy_$v.so; done); do
  export HWY_LIB=$R/highway-rope-ppo_amd/hwy/$lib
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats --kernel-include-regex "ppo_" \
    -d $R/gpurun_out/kt/$lib -o run --output-format csv \
    -- python3 $R/tools/probe_ppo_time.py 256 3 ${MB:-16384} > $R/gpurun_out/kt/$lib.log 2>&1 || { echo "kt $lib failed"; tail -3 $R/gpurun_out/kt/$lib.log; exit 1; }
  f=$(find $R/gpurun_out/kt/$lib -name "*kernel_stats.csv" | head -1)
  echo "== $lib"; python3 $R/tools/summarize_stats.py "$f" 4
done
