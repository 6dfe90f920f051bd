# ppo_wgrad partition A/B (development aid): fused-update tests, then the minibatch step time
# with the balanced partition and with one workgroup per (tile, slice) (HWY_WG_WPX=26)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_ppo_fused_gpu.py tests/test_dist_fused_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/wg_tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/wg_tests.log; exit 1; }
tail -2 gpurun_out/wg_tests.log
for wpx in 0 26; do for mb in 16384 4096; do
  HWY_WG_WPX=$wpx timeout -k 10 60 python -u tools/probe_ppo_time.py 256 5 $mb | sed "s/^/wpx=$wpx mb=$mb /" || exit 1
done; done
cd /tmp
for wpx in 0 26; do
HWY_WG_WPX=$wpx timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/wg$wpx -o run -- python3 $R/tools/probe_ppo_time.py 256 3 16384 > $R/gpurun_out/wg$wpx.log 2>&1 || exit 1
python3 $R/tools/summarize_stats.py $R/gpurun_out/wg$wpx/run_kernel_stats.csv 5
done
