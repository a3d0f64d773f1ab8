# Round 5, first GPU iteration: where the default-limit configs[3] scatter's extra reads come from
# (admission lookup off / XCD-aware tile ranges, times + FETCH/WRITE + L2 hit/miss), and the select pass's
# occupancy (waves-per-EU hint) on SSB Q4.2 / Q3.2 / Q2.2.
set -o pipefail
mkdir -p gpurun_out
HC="--workload highcard-default --segments 40"
SWEEP="none PINOT_AMD_XCD_REMAP=1 PINOT_AMD_DIAG_ADMIT_OFF=1" ARGS="$HC" STEPS=5 timeout -k 10 400 bash scripts/gpu_sweep.sh || exit 1
cp gpurun_out/sweep.txt gpurun_out/r5_sweep_hcdef.txt
SWEEP="none PINOT_AMD_XCD_REMAP=1" ARGS="--workload highcard --segments 40" STEPS=5 timeout -k 10 300 bash scripts/gpu_sweep.sh || exit 1
cp gpurun_out/sweep.txt gpurun_out/r5_sweep_hc.txt
CASES="base||$HC;remap|PINOT_AMD_XCD_REMAP=1|$HC;off|PINOT_AMD_DIAG_ADMIT_OFF=1|$HC" \
  SETS="FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum" timeout -k 10 900 bash scripts/pmc_ab.sh > gpurun_out/r5_pmc_hcdef.txt || exit 1
echo pmc done
: > gpurun_out/r5_sweep_ssb_wpe.txt
for q in 11 7 4; do
  SWEEP="none PINOT_AMD_WAVES_PER_EU=5 PINOT_AMD_WAVES_PER_EU=6" ARGS="--workload ssb --query-index $q" STEPS=10 timeout -k 10 300 bash scripts/gpu_sweep.sh || exit 1
  cat gpurun_out/sweep.txt >> gpurun_out/r5_sweep_ssb_wpe.txt
done
