#!/bin/bash
# Per-section shader clocks (profiling build, make prof) of ppo_rows / ppo_wgrad, ppo_rowsT and
# hwy_step at the bench shapes.  Run from the repo root on the GPU box.
set -o pipefail
mkdir -p gpurun_out/r3
O=gpurun_out/r3/sections.log
: > $O
timeout -k 10 120 python -u tools/probe_ppo_sections.py 256 16384 >> $O 2>&1 && \
HWY_ROWS_T=1 timeout -k 10 120 python -u tools/r3/probe_rowsT_sections.py 256 16384 >> $O 2>&1 && \
timeout -k 10 120 python -u tools/probe_sections.py 4096 >> $O 2>&1
rc=$?
cat $O
exit $rc
