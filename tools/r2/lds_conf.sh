# LDS bank-conflict cycles of ppo_rows per library variant (development aid)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
for v in "$@"; do
  L=$R/highway-rope-ppo_amd/hwy/libhwy_$v.so; [ $v = base ] && L=$R/highway-rope-ppo_amd/hwy/libhwy.so
  HWY_LIB=$L timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS --kernel-include-regex ppo_rows -d $R/gpurun_out/ldsc_$v -o run --output-format csv -- python3 $R/tools/probe_ppo_time.py 256 2 16384 > $R/gpurun_out/ldsc_$v.log 2>&1 || { echo "$v failed"; exit 1; }
  echo "== $v"; python3 $R/tools/pmc_table.py $R/gpurun_out/ldsc_$v | grep -E "SQ_"
done
