#!/bin/bash
# ppo_rows_c wave-priority sweep (dev build: HWY_ROWS_PRIO)
set -o pipefail
D=$PWD/highway-rope-ppo_amd/hwy/libhwy_dev.so
for p in 0 1 2 3 0 1 2 3; do
  HWY_LIB=$D HWY_ROWS_PRIO=$p timeout -k 10 60 python -u tools/probe_ppo_time.py 256 10 16384 | sed "s/^/prio=$p /" || exit 1
done
