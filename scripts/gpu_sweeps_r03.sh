# Round-3 knob sweeps: non-temporal loads on configs[1]; select-pass pipeline depth / occupancy on the
# SSB selection-vector queries (Q1.2, Q4.2); results in gpurun_out/sweep_*.txt.
set -o pipefail
SWEEP="none PINOT_AMD_NT_LOADS=1" ARGS="--segments 100" STEPS=20 bash scripts/gpu_sweep.sh && cp gpurun_out/sweep.txt gpurun_out/sweep_scan_nt.txt || exit 1
for qi in 1 11; do
  SWEEP="none PINOT_AMD_PREFETCH=2 PINOT_AMD_PREFETCH=4 PINOT_AMD_PREFETCH=6 PINOT_AMD_PREFETCH=8 PINOT_AMD_NT_LOADS=1 PINOT_AMD_SELECT=never" \
    ARGS="--workload ssb --query-index $qi" STEPS=10 bash scripts/gpu_sweep.sh && cp gpurun_out/sweep.txt gpurun_out/sweep_ssb$qi.txt || exit 1
done
