export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 || { echo BENCHFAIL; tail -20 gpurun_out/bench.log; exit 1; }
grep '^{' gpurun_out/bench.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu-baseline > gpurun_out/bench_prof.log 2>&1 || { echo PROFFAIL; exit 1; }
python3 tools/summarize_stats.py $(ls gpurun_out/prof/*/run_kernel_stats.csv gpurun_out/prof/run_kernel_stats.csv 2>/dev/null | head -1) 10
