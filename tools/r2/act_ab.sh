# rollout time and rocprofv3 kernel averages per library variant (development aid):
#   act_ab.sh tag ...   (highway-rope-ppo_amd/hwy/libhwy_<tag>.so; "base" = libhwy.so)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
for v in "$@"; do
  L=$R/highway-rope-ppo_amd/hwy/libhwy_$v.so; [ $v = base ] && L=$R/highway-rope-ppo_amd/hwy/libhwy.so
  SPLIT=0 HWY_LIB=$L timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/act_$v -o run -- python3 $R/tools/r2/split_probe.py 4096 128 5 > $R/gpurun_out/act_$v.log 2>&1 || { echo "$v failed"; tail -5 $R/gpurun_out/act_$v.log; exit 1; }
  echo "== $v: $(grep 'single stream' $R/gpurun_out/act_$v.log)"
  python3 $R/tools/summarize_stats.py $R/gpurun_out/act_$v/run_kernel_stats.csv 6 | grep -E "ppo_act|hwy_step"
done
