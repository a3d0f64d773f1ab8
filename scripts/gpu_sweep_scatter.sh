# Scatter flush cadence sweep on configs[3] (SET limit) and highcard-default (admission).
set -o pipefail
SWEEP="none PINOT_AMD_FLUSH_EVERY=2 PINOT_AMD_FLUSH_EVERY=3 PINOT_AMD_FLUSH_EVERY=4" ARGS="--workload highcard" STEPS=10 bash scripts/gpu_sweep.sh && cp gpurun_out/sweep.txt gpurun_out/sweep_hc_flush.txt || exit 1
SWEEP="none PINOT_AMD_FLUSH_EVERY=2 PINOT_AMD_FLUSH_EVERY=4 PINOT_AMD_FLUSH_EVERY=8" ARGS="--workload highcard-default" STEPS=5 bash scripts/gpu_sweep.sh && cp gpurun_out/sweep.txt gpurun_out/sweep_hcdef_flush.txt
