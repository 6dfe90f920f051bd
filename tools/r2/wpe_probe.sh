# ppo_rows occupancy A/B (development aid): 16-row tiles compiled for 1 or 2 workgroups per CU
export TMPDIR=/tmp
for i in 1 2; do for v in base wpe4; do
  L=highway-rope-ppo_amd/hwy/libhwy.so; [ $v = wpe4 ] && L=highway-rope-ppo_amd/hwy/libhwy_wpe4.so
  for rt in 16 32; do
    HWY_ROWS_RT=$rt HWY_LIB=$L timeout -k 10 60 python -u tools/probe_ppo_time.py 256 5 16384 | sed "s/^/$v rt$rt /" || exit 1
  done
  HWY_LIB=$L timeout -k 10 60 python -u tools/probe_ppo_time.py 256 5 4096 | sed "s/^/$v 4096 /" || exit 1
done; done
