# The round's measurement set in one GPU call: tools/r2/measure.sh (bench lines for configs 1-4,
# rocprofv3 kernel stats, hwy_step PMC) and the PMC traffic of the minibatch step at 16,384 and
# 4,096 rows (tools/pmc_ppo_traffic.sh -> profiles/ppo_step_pmc*.json)
set -u
bash tools/r2/measure.sh || exit 1
for mb in 16384 4096; do
  echo "[measure] pmc ppo $mb"
  MB=$mb bash tools/pmc_ppo_traffic.sh > gpurun_out/r2m/pmc_ppo_$mb.log 2>&1 || { tail -20 gpurun_out/r2m/pmc_ppo_$mb.log; exit 1; }
  grep -E "hbm_side_bytes_per_step" gpurun_out/r2m/pmc_ppo_$mb.log
done
mkdir -p gpurun_out/r2m/pmc_json && cp profiles/ppo_step_pmc*.json gpurun_out/r2m/pmc_json/
echo "[measure] all done"
