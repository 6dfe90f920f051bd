# register loss head at 16-row tiles (development A/B): timing at 4,096 rows (H 256) and at
# 8,192 rows with H 384 / 512 (16-row tiles there), same box
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
for i in 1 2; do for v in base reg16; do
  L=$R/highway-rope-ppo_amd/hwy/libhwy_$v.so; [ $v = base ] && L=$R/highway-rope-ppo_amd/hwy/libhwy.so
  for hm in "256 4096" "384 8192" "512 8192"; do
    set -- $hm
    HWY_LIB=$L timeout -k 10 60 python3 $R/tools/probe_ppo_time.py $1 3 $2 | sed "s/^/$v mb=$2 /" || exit 1
  done
done; done
