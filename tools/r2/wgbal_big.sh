# ppo_wgrad balanced partition at H 384 / 512 (configs[4] learner shapes, development A/B)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_ppo_fused_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/wgbal_big_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/wgbal_big_tests.log; exit 1; }
tail -1 gpurun_out/wgbal_big_tests.log
cd /tmp
for hm in "384 32768" "512 32768"; do set -- $hm; for b in 1 0; do
  HWY_WG_BAL=$b timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/wgb_$b -o run -- python3 $R/tools/probe_ppo_time.py $1 2 $2 > $R/gpurun_out/wgb_$b.log 2>&1 || { echo "bal=$b failed"; tail -5 $R/gpurun_out/wgb_$b.log; exit 1; }
  echo "== H=$1 mb=$2 bal=$b: $(grep 'us per' $R/gpurun_out/wgb_$b.log)"
  python3 $R/tools/summarize_stats.py $R/gpurun_out/wgb_$b/run_kernel_stats.csv 4 | grep -E "ppo_wgrad|ppo_wsum|ppo_rows"
done; done
