#!/bin/bash
# Copy the judged artefacts of tools/r2/measure.sh from gpurun_out/r2m into profiles/r2 (and the
# PMC summaries bench.py reads into profiles/).
set -e
S=${1:-gpurun_out/r2m}
D=profiles/r2
mkdir -p $D
for f in $S/bench_c*.json; do cp "$f" $D/; done
for c in 1 2; do
  cp $S/kernel_stats_c$c.txt $D/bench_kernel_stats_c${c}_top.txt
  grep '^{' $S/bench_prof_c$c.log > $D/bench_under_rocprof_c$c.json || true
done
python3 tools/summarize_stats.py $(ls $S/prof_c1/run_results.db $S/prof_c1/*/run_results.db 2>/dev/null | head -1) 40 > $D/bench_kernel_stats_c1.txt
cp $S/hwy_step_valu.json profiles/hwy_step_valu.json
cp $S/hwy_step_pmc.json profiles/hwy_step_pmc.json
cp profiles/hwy_step_valu.json profiles/hwy_step_pmc.json $D/
ls -la $D
