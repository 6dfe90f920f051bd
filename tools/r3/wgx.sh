#!/bin/bash
# ppo_wgrad timing-only experiments: kernel-trace stats of the product library and the wgx
# variants (HWY_WG_EXP builds) at 16,384 rows
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/wgx
for lib in libhwy.so libhwy_wgx1.so libhwy_wgx2.so libhwy_wgx3.so libhwy_wgx4.so; do
  export HWY_LIB=$R/highway-rope-ppo_amd/hwy/$lib
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats --kernel-include-regex "ppo_" \
    -d $R/gpurun_out/wgx/$lib -o run --output-format csv \
    -- python3 $R/tools/probe_ppo_time.py 256 3 16384 > $R/gpurun_out/wgx/$lib.log 2>&1 || { echo "kt $lib failed"; tail -3 $R/gpurun_out/wgx/$lib.log; exit 1; }
  f=$(find $R/gpurun_out/wgx/$lib -name "*kernel_stats.csv" | head -1)
  echo "== $lib"; python3 $R/tools/summarize_stats.py "$f" 6
done
