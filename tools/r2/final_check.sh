# Round-end rehearsal on one MI355X: the GPU test suite, smoke(), the default bench line and its
# rocprofv3 kernel statistics
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/final
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final/gpu_tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/final/gpu_tests.log; exit 1; }
tail -1 gpurun_out/final/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final/smoke.log 2>&1 || { echo SMOKEFAIL; tail -20 gpurun_out/final/smoke.log; exit 1; }
tail -1 gpurun_out/final/smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/final/bench.log 2>&1 || { echo BENCHFAIL; tail -20 gpurun_out/final/bench.log; exit 1; }
grep '^{' gpurun_out/final/bench.log | cut -c1-300
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/final/prof -o run -- python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/final/bench_prof.log 2>&1 || { echo PROFFAIL; exit 1; }
python3 $R/tools/summarize_stats.py $R/gpurun_out/final/prof/run_kernel_stats.csv 8
