#!/bin/bash
# hwy_ppo_step (one-launch gradient sums + Adam) against the two-call step: the bit-equality test,
# then interleaved minibatch-step times at configs[1] / configs[4]-like shapes.
set -o pipefail
mkdir -p gpurun_out/wsa
timeout -k 10 600 python -u -m pytest tests/test_ppo_fused_gpu.py -x -v --timeout 300 --timeout-method thread \
  -k "single_call or matches_torch_update or replays_reference or adam" > gpurun_out/wsa/tests.log 2>&1
rc=$?; tail -3 gpurun_out/wsa/tests.log; [ $rc -eq 0 ] || exit $rc
for shp in 256:16384:60 256:32768:120 384:32768:240; do
  IFS=: read Hd mb S <<< "$shp"
  for rep in 1 2 3; do
    for sp in 1 0; do
      HWY_SPLIT_STEP=$sp timeout -k 10 90 python -u tools/probe_ppo_time.py $Hd 10 $mb $S \
        | sed "s/^/split=$sp H=$Hd mb=$mb S=$S /" || exit 1
    done
  done
done
