#!/bin/bash
# kernel-trace stats of the PPO minibatch step at configs[4]'s shapes, product vs variants
# (SHAPES: "H reps rows S" entries separated by commas)
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/kts
IFS=, read -ra SH <<< "${SHAPES:-384 2 32768 240,512 2 32768 120}"
for shape in "${SH[@]}"; do
  for lib in libhwy.so $(for v in $VARS; do echo libhwy_$v.so; done); do
    export HWY_LIB=$R/highway-rope-ppo_amd/hwy/$lib
    tag=$(echo "$shape $lib" | tr ' ' '_')
    timeout -s KILL 120 rocprofv3 --kernel-trace --stats --kernel-include-regex "ppo_" \
      -d $R/gpurun_out/kts/$tag -o run --output-format csv \
      -- python3 $R/tools/probe_ppo_time.py $shape > $R/gpurun_out/kts/$tag.log 2>&1 || { echo "kt $tag failed"; tail -3 $R/gpurun_out/kts/$tag.log; exit 1; }
    f=$(find $R/gpurun_out/kts/$tag -name "*kernel_stats.csv" | head -1)
    echo "== $shape $lib"; python3 $R/tools/summarize_stats.py "$f" 4 | grep ppo_ | cut -c1-100
  done
done
