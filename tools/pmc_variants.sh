#!/bin/bash
# PMC comparison of hwy_step variants (development aid): pmc_variants.sh v1 v2 ...
set -e
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/pmcv
timeout -k 10 60 rocprofv3 -L > $R/gpurun_out/pmcv/list.txt 2>&1
pick() { for c in "$@"; do grep -qw "$c" $R/gpurun_out/pmcv/list.txt && echo -n "$c "; done; }
S1=$(pick SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM)
S2=$(pick SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_WAVES SQC_ICACHE_MISSES_DUPLICATE)
echo "sets: [$S1] [$S2]"
for v in "$@"; do
  for set in "$S1" "$S2"; do
    [ -z "$set" ] && continue
    tag=$(echo $set | cut -c1-6)
    timeout -k 10 120 rocprofv3 --pmc $set --kernel-include-regex hwy_step -d $R/gpurun_out/pmcv/${v}_$tag -o run --output-format csv -- python3 $R/tools/probe_variant.py $R/highway-rope-ppo_amd/hwy/libhwy_exp_$v.so 4096
  done
done
