# ppo_wgrad balanced partition check (development aid): fused-update tests, then rocprofv3
# kernel averages with the balanced partition and with HWY_WG_BAL=0, same box
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_ppo_fused_gpu.py tests/test_dist_fused_gpu.py tests/test_agent_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/wgbal_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/wgbal_tests.log; exit 1; }
tail -1 gpurun_out/wgbal_tests.log
cd /tmp
for mb in 16384 32768; do for i in 1 2; do for b in 1 0; do
  HWY_WG_BAL=$b timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/wgbal_$b -o run -- python3 $R/tools/probe_ppo_time.py 256 3 $mb > $R/gpurun_out/wgbal_$b.log 2>&1 || { echo "bal=$b failed"; tail -5 $R/gpurun_out/wgbal_$b.log; exit 1; }
  echo "== mb=$mb bal=$b: $(grep 'us per' $R/gpurun_out/wgbal_$b.log)"
  python3 $R/tools/summarize_stats.py $R/gpurun_out/wgbal_$b/run_kernel_stats.csv 4 | grep -E "ppo_wgrad|ppo_wsum"
done; done; done
