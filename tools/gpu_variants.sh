#!/bin/bash
# rocprofv3 kernel stats of probe_ppo_time.py per library variant (development aid):
#   gpu_variants.sh <kernel regex> lib1 lib2 ...   (libs under highway-rope-ppo_amd/hwy/)
R=$(pwd); K=$1; shift
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/var
for v in "$@"; do
  HWY_LIB=$R/highway-rope-ppo_amd/hwy/$v timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $R/gpurun_out/var/$v -o run -- python3 $R/tools/probe_ppo_time.py 256 3 > $R/gpurun_out/var/$v.log 2>&1 || { echo "$v failed"; tail -5 $R/gpurun_out/var/$v.log; exit 1; }
  echo "== $v: $(grep 'us per' $R/gpurun_out/var/$v.log)"
  python3 $R/tools/summarize_stats.py $R/gpurun_out/var/$v/run_kernel_stats.csv 6 | grep -E "$K|ppo_" 
done
