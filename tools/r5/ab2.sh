#!/bin/bash
# round-5 A/B 2: ppo_act_c at one workgroup per CU with a 4-deep ring (product) vs the 2-deep
# two-per-CU budget (actd2); the IDM pow as one branch-free sequence (product) vs hm_powf (oldpow)
set -o pipefail
MODE=act VARS="actd2" TESTS=1 ROWS="4096 8192" REPS=2 bash tools/ab.sh > gpurun_out/ab2_act.log 2>&1 || { tail -20 gpurun_out/ab2_act.log; exit 1; }
grep -E "passed|failed|==|ppo_act" gpurun_out/ab2_act.log
MODE=step VARS="oldpow nosatpre" TESTS=1 ENVS="4096 16384" REPS=3 bash tools/ab.sh > gpurun_out/ab2_step.log 2>&1 || { tail -20 gpurun_out/ab2_step.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ab2_step.log
MODE=pmc VARS="oldpow nosatpre" REPS=1 bash tools/ab.sh > gpurun_out/ab2_pmc.log 2>&1 || { tail -20 gpurun_out/ab2_pmc.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ab2_pmc.log
