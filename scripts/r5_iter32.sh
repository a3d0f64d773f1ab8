# Round 5, thirty-second GPU iteration: configs[3] (default limit and untrimmed) with / without the scatter self-check,
# interleaved (PINOT_AMD_SCATTER_CHECK=0 turns it off).
set -o pipefail
mkdir -p gpurun_out
SWEEP="none PINOT_AMD_SCATTER_CHECK=0 none PINOT_AMD_SCATTER_CHECK=0" ARGS="--workload highcard-default" STEPS=10 timeout -k 10 600 bash scripts/gpu_sweep.sh || exit 1
cp gpurun_out/sweep.txt gpurun_out/r5_sweep_hcdef_selfcheck.txt
SWEEP="none PINOT_AMD_SCATTER_CHECK=0" ARGS="--workload highcard" STEPS=10 timeout -k 10 600 bash scripts/gpu_sweep.sh || exit 1
cp gpurun_out/sweep.txt gpurun_out/r5_sweep_hc_selfcheck.txt
