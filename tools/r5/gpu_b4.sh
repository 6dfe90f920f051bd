#!/bin/bash
# the last intermediate-recipe cell, then the bench line's recipe (T = 32) on the final kernels
set -o pipefail
PART=B CELLS="shuffled_rankpe:256" OUT=gpurun_out/r5_reward TAG=pe2 bash tools/reward.sh &&
PART=A OUT=gpurun_out/r5_reward TAG=a bash tools/reward.sh
