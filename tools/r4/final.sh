#!/bin/bash
# Round-4 final record on the final tree: GPU tests + smoke + default bench, then the bench lines of
# configs 1-4 and the rocprofv3 kernel stats of the configs[1] / configs[2] benches (tools/r4/measure.sh).
set -o pipefail
bash tools/r4/gpu_tests.sh && OUT=gpurun_out/r4m bash tools/r4/measure.sh
