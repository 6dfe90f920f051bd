#!/bin/bash
# 16-row tiles at 16 waves (4 per SIMD) against 8: parity tests, then the 4,096-row step
set -o pipefail
export PROBE_KT=1
VARS="nw16" MODE=ppo SHAPES="256:4096:60" REPS=3 bash tools/ab.sh 2>&1 | grep -v amdgpu.ids
