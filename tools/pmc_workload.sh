#!/bin/bash
# PMC evidence for one bench workload (bench.py --config C), in separate rocprofv3 passes
# (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE never in one pass):
#   hwy_step   FETCH_SIZE, WRITE_SIZE (calibrated against known-byte kernels) and the
#              instruction counts SQ_INSTS_{VALU,SALU,LDS,BRANCH} + SQ_WAVES
#   PPO step   FETCH_SIZE, WRITE_SIZE of ppo_rows / ppo_wgrad / ppo_wsum / ppo_adam at the
#              workload's minibatch (rows = E x T / 32) and state width S = N x F_out
# -> profiles/hwy_step_pmc_E*_N*_F*.json, profiles/hwy_step_valu_E*_N*_F*.json,
#    profiles/ppo_step_pmc_<rows>_S*_H*.json  (bench.py attaches them by those keys)
#   CONFIG=2 bash tools/pmc_workload.sh        (run from the repo root on the GPU box)
set -u
R=$(pwd)
C=${CONFIG:-2}
read E N F T <<<"$(python3 -c "
import sys; sys.path.insert(0, '.')
from bench import CONFIGS
w = CONFIGS[$C]; print(w['envs'], w['obs'], 8 if w['pe'] in ('rank', 'dist') else 4, w['rollout'])")"
S=$((N * F)); H=${H:-256}; MB=$((E * T / 32))
O=$R/gpurun_out/pmc_c$C
mkdir -p $O
echo "config $C: E=$E N=$N F=$F S=$S rows=$MB H=$H"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/calib/pmc_calib.hip \
  -o tools/calib/libpmc_calib.so || exit 1
cd /tmp && export TMPDIR=/tmp
run() {  # run <tag> <counters> <kernel regex> <command...>
  local tag=$1 cnt=$2 re=$3; shift 3
  timeout -s KILL 150 rocprofv3 --pmc $cnt --kernel-include-regex "$re" -d $O/$tag -o run \
    --output-format csv -- "$@" > $O/$tag.log 2>&1 || { echo "pass $tag failed"; tail -5 $O/$tag.log; exit 1; }
  echo "pass $tag ok"
}
export PMC_CONFIG=$C
run fetch FETCH_SIZE "hwy_step|calib" python3 $R/tools/calib/pmc_step.py
run write WRITE_SIZE "hwy_step|calib" python3 $R/tools/calib/pmc_step.py
run valu "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVES" "hwy_step" \
  python3 $R/tools/calib/pmc_step.py
mkdir -p $O/ppo
run ppo/FETCH_SIZE FETCH_SIZE "ppo_(rows|wgrad|wsum|adam)" python3 $R/tools/probe_ppo_time.py $H 2 $MB $S
run ppo/WRITE_SIZE WRITE_SIZE "ppo_(rows|wgrad|wsum|adam)" python3 $R/tools/probe_ppo_time.py $H 2 $MB $S
cd $R
python3 tools/calib/pmc_summarize.py $O $E $N $F > /dev/null && \
python3 tools/calib/valu_summarize.py $O/valu $N $F > /dev/null && \
python3 tools/calib/ppo_traffic_summarize.py $O/ppo $MB $S $H | grep hbm_side
ls -1 profiles/*E${E}_N${N}* profiles/ppo_step_pmc_${MB}_S${S}_H${H}.json || true  # (written where the summaries run; gpurun merges only gpurun_out/)
