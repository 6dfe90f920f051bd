# minibatch-step time of library variants (development A/B): variants.sh rows tag1 tag2 ...
export TMPDIR=/tmp
MB=$1; shift
for v in "" "$@"; do
  L=highway-rope-ppo_amd/hwy/libhwy${v:+_$v}.so
  HWY_LIB=$L timeout -k 10 60 python -u tools/probe_ppo_time.py 256 5 $MB | sed "s/^/${v:-base} /" || exit 1
done
