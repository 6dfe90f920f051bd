# ppo_wgrad balanced-partition fill price A/B (development aid): rocprofv3 kernel averages of
# tools/probe_ppo_time.py at 16,384 rows for several HWY_WG_FILL values on one box
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
for f in "$@"; do
  HWY_WG_FILL=$f timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/fill_$f -o run -- python3 $R/tools/probe_ppo_time.py 256 3 16384 > $R/gpurun_out/fill_$f.log 2>&1 || { echo "$f failed"; exit 1; }
  echo "== fill $f: $(grep 'us per' $R/gpurun_out/fill_$f.log)"
  python3 $R/tools/summarize_stats.py $R/gpurun_out/fill_$f/run_kernel_stats.csv 4 | grep -E "ppo_wgrad|ppo_wsum"
done
