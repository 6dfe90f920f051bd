# rocprofv3 kernel averages of tools/probe_ppo_time.py per library variant (development aid):
#   lib_ab.sh <rows> tag ...   (highway-rope-ppo_amd/hwy/libhwy_<tag>.so; "base" = libhwy.so)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
MB=$1; shift
cd /tmp
for v in "$@"; do
  L=$R/highway-rope-ppo_amd/hwy/libhwy_$v.so; [ $v = base ] && L=$R/highway-rope-ppo_amd/hwy/libhwy.so
  HWY_LIB=$L timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ab_$v -o run -- python3 $R/tools/probe_ppo_time.py 256 3 $MB > $R/gpurun_out/ab_$v.log 2>&1 || { echo "$v failed"; tail -5 $R/gpurun_out/ab_$v.log; exit 1; }
  echo "== $v: $(grep 'us per' $R/gpurun_out/ab_$v.log)"
  python3 $R/tools/summarize_stats.py $R/gpurun_out/ab_$v/run_kernel_stats.csv 4 | grep ppo_
done
