export TMPDIR=/tmp
for v in "" _NOFENCE _NOREDUCE; do
  echo "variant [$v]"; HWY_LIB=$PWD/highway-rope-ppo_amd/hwy/libhwy$v.so timeout -k 10 120 python3 tools/probe_ppo_time.py 256 5 || exit 1
done
timeout -k 10 120 python3 tools/probe_ppo_sections.py 256 || exit 1
