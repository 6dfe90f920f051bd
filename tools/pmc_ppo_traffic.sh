#!/bin/bash
# HBM-side traffic of the fused PPO minibatch step (ppo_rows / ppo_wgrad / ppo_wsum / ppo_adam):
# two rocprofv3 passes (FETCH_SIZE, WRITE_SIZE) over tools/probe_ppo_time.py at the bench
# minibatch, then tools/calib/ppo_traffic_summarize.py -> profiles/ppo_step_pmc.json.
R=$(pwd)
MB=${MB:-16384}  # minibatch rows (the bench's configs[1] default: 4096 envs x 128 steps / 32)
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/pmc_ppo
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex "ppo_(rows|wgrad|wsum|adam)" \
    -d $R/gpurun_out/pmc_ppo/$c -o run --output-format csv -- python3 $R/tools/probe_ppo_time.py 256 2 $MB \
    > $R/gpurun_out/pmc_ppo/$c.log 2>&1 || { echo "pass $c failed"; tail -5 $R/gpurun_out/pmc_ppo/$c.log; exit 1; }
done
cd $R && python3 tools/calib/ppo_traffic_summarize.py gpurun_out/pmc_ppo $MB
