#!/bin/bash
# configs[4]'s hidden sweep at the lockstep recipe (E 4096, T 128, 320k episodes): sorted h384 / h512
set -o pipefail
COND=sorted HID=384 RUN_LIMIT=560 OUT=gpurun_out/r3_reward/sorted_h384_e4096_t128 bash tools/r3/reward_cell.sh && \
COND=sorted HID=512 RUN_LIMIT=560 OUT=gpurun_out/r3_reward/sorted_h512_e4096_t128 bash tools/r3/reward_cell.sh
