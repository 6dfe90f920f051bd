# hwy_step per library variant (development aid): step_ab.sh tag ... ("base" = libhwy.so)
export TMPDIR=/tmp
for v in "$@"; do
  L=highway-rope-ppo_amd/hwy/libhwy_$v.so; [ $v = base ] && L=highway-rope-ppo_amd/hwy/libhwy.so
  HWY_LIB=$L timeout -k 10 60 python -u tools/probe_step.py 4096 | sed "s/^/$v /" || exit 1
done
