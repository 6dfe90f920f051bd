bash tools/r4/gpu_tests.sh && mkdir -p gpurun_out/r4m && cd /tmp && export TMPDIR=/tmp && cd - >/dev/null && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4m/prof_c1 -o run -- python3 bench.py --config 1 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r4m/bench_prof_c1.log 2>&1 && \
S=$(ls gpurun_out/r4m/prof_c1/run_kernel_stats.csv gpurun_out/r4m/prof_c1/*/run_kernel_stats.csv 2>/dev/null | head -1) && \
python3 tools/summarize_stats.py "$S" 16 > gpurun_out/r4m/kernel_stats_c1.txt && head -12 gpurun_out/r4m/kernel_stats_c1.txt
