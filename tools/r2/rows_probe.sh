# ppo_rows A/B (development aid): fused-update tests, then the minibatch step time and the
# rocprofv3 kernel averages at the bench minibatch (16,384 rows) and at 4,096 rows
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_ppo_fused_gpu.py tests/test_dist_fused_gpu.py tests/test_agent_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/rows_tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/rows_tests.log; exit 1; }
tail -2 gpurun_out/rows_tests.log
for mb in 16384 4096; do
  timeout -k 10 60 python -u tools/probe_ppo_time.py 256 5 $mb | sed "s/^/mb=$mb /" || exit 1
done
cd /tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/rowsprof -o run -- python3 $R/tools/probe_ppo_time.py 256 3 16384 > $R/gpurun_out/rowsprof.log 2>&1 || exit 1
python3 $R/tools/summarize_stats.py $R/gpurun_out/rowsprof/run_kernel_stats.csv 5
