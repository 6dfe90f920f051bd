#!/bin/bash
# A/B of the hwy_step wave-mask rework: prev (before it), product, nbloop (lane masks by the
# select loop), omloop (pair list from the 64-bit mask), r4ish (both)
set -o pipefail
VARS="prev nbloop omloop r4ish" MODE=pmc REPS=1 bash tools/ab.sh 2>&1 | grep launches &&
VARS="prev nbloop omloop r4ish" MODE=step REPS=3 ENVS="4096 16384" bash tools/ab.sh 2>&1 | grep env-steps
