#!/bin/bash
# full GPU suite + smoke + default bench, then the clock / MFMA-busy PMC comparison
set -o pipefail
bash tools/r3/gpu_tests.sh && bash tools/r3/pmc_clock.sh
