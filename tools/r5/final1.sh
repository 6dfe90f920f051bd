#!/bin/bash
# Round-5 final record, part 1: GPU tests + smoke + default bench, then the rocprofv3 kernel stats
# of the configs[1] / configs[2] benches (tools/measure.sh)
set -o pipefail
OUT=gpurun_out/r5m PART=tests bash tools/measure.sh && OUT=gpurun_out/r5m PART=prof bash tools/measure.sh
