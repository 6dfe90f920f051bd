export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ppo_fused_gpu.py -x -q --timeout 120 --timeout-method thread -k "gradient_matches_autograd or update_matches" > gpurun_out/rt_tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/rt_tests.log; exit 1; }
tail -2 gpurun_out/rt_tests.log
for rt in 16 32; do for mb in 16384 8192; do
  HWY_ROWS_RT=$rt timeout -k 10 60 python -u tools/probe_ppo_time.py 256 5 $mb | sed "s/^/rt=$rt mb=$mb /" || exit 1
done; done
cd /tmp
for rt in 16 32; do
HWY_ROWS_RT=$rt timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/rt$rt -o run -- python3 $GRAFT_REPO_ROOT/tools/probe_ppo_time.py 256 3 16384 > $GRAFT_REPO_ROOT/gpurun_out/rt$rt.log 2>&1 || exit 1
python3 $GRAFT_REPO_ROOT/tools/summarize_stats.py $GRAFT_REPO_ROOT/gpurun_out/rt$rt/run_kernel_stats.csv 6
done
