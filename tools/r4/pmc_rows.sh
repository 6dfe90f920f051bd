#!/bin/bash
# PMC passes over the row kernel of each library (ppo_rows_r in libhwy.so, ppo_rows_c64 in
# libhwy_c64.so) at the bench minibatch; the instruction-cache pass is allowed to fail.
R=$(pwd); H=$R/highway-rope-ppo_amd/hwy; O=$R/gpurun_out/pmcr; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for lib in libhwy_roll.so libhwy.so libhwy_c64.so; do
  i=0
  for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
             "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVES" \
             "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
             "SQC_ICACHE_MISSES SQC_ICACHE_HITS"; do
    i=$((i+1))
    HWY_LIB=$H/$lib timeout -s KILL 90 rocprofv3 --pmc $set --kernel-include-regex ppo_rows -d $O/${lib%.so}_$i -o run \
      --output-format csv -- python3 $R/tools/probe_ppo_time.py 256 2 16384 > $O/${lib%.so}_$i.log 2>&1 || { echo "pass $i on $lib failed"; tail -3 $O/${lib%.so}_$i.log; [ $i -eq 4 ] || exit 1; }
  done
done
O=$O python3 - <<'PY'
import csv, glob, collections, os
O = os.environ.get("O", "gpurun_out/pmcr")
for lib in ("libhwy_roll", "libhwy", "libhwy_c64"):
    tot = collections.defaultdict(float); n = collections.defaultdict(int)
    for f in glob.glob(f"{O}/{lib}_*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    print(lib, {k: f"{v:.4g}" for k, v in sorted(tot.items())})
PY
cd $R && bash tools/r4/ab_rows_r2.sh
