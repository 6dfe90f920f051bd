# ppo_rows change check (development aid): the fused-update / agent / distributed GPU tests, then
# the minibatch step time and rocprofv3 kernel averages at 16,384 and 4,096 rows
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_ppo_fused_gpu.py tests/test_agent_gpu.py tests/test_dist_fused_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/rows_check.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/rows_check.log; exit 1; }
tail -2 gpurun_out/rows_check.log
bash tools/r2/lib_ab.sh 16384 base || exit 1
bash tools/r2/lib_ab.sh 4096 base || exit 1
