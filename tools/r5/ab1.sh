set -o pipefail
# round-5 A/B: product (pre-gathered rows) vs XCD-clustered row tiles vs ring depth 8 (16-row tiles)
MODE=ppo VARS="xcd d8" SHAPES="256:4096:60 256:16384:60" REPS=3 bash tools/ab.sh > gpurun_out/ab1_ppo.log 2>&1 || { tail -20 gpurun_out/ab1_ppo.log; exit 1; }
cat gpurun_out/ab1_ppo.log
MODE=kt VARS="xcd d8" MB=4096 REPS=1 bash tools/ab.sh > gpurun_out/ab1_kt.log 2>&1 || { tail -20 gpurun_out/ab1_kt.log; exit 1; }
cat gpurun_out/ab1_kt.log
timeout -k 10 300 python -u bench.py --steps 8 --warmup 3 --no-cpu-baseline > gpurun_out/bench_pk.json 2> gpurun_out/bench_pk.err || { tail -5 gpurun_out/bench_pk.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/bench_pk.json').read().strip().splitlines()[-1]); r=d['roofline']
print(d['value'], r['avg_launch_us'], json.dumps(r['per_kernel']))"
