#!/bin/bash
# kernel-trace average of hwy_step_kernel: product vs variants ($VARS), c1 shape at 4096 envs and
# the 30-row PE shapes at 16,384 ($PES)
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/kts
run() {  # lib tag args...
  local lib=$1 tag=$2; shift 2
  local d=$R/gpurun_out/kts/${lib%.so}_${tag}_$rep
  HWY_LIB=$R/highway-rope-ppo_amd/hwy/$lib timeout -s KILL 90 rocprofv3 --kernel-trace --stats \
    -d $d -o run --output-format csv -- python3 "$@" > $d.log 2>&1 || { echo "kt $lib $tag failed"; tail -3 $d.log; return 1; }
  local s=$(find $d -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv
for r in csv.DictReader(open('$s')):
    if 'hwy_step' in r['Name']:
        print('$lib', '$tag', r['Name'][:32], r['Calls'], '%.1f us' % (float(r['AverageNs'])/1e3))"
}
for rep in 1 2; do
  for lib in libhwy.so $(for v in $VARS; do echo libhwy_$v.so; done); do
    run $lib c1 $R/tools/probe_step.py 4096 || exit 1
    for p in ${PES:-rope}; do run $lib $p $R/tools/r3/probe_step_pe.py $p 16384 || exit 1; done
  done
done
