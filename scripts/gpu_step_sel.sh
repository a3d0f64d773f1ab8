# Round-3 selective-plan check: the GPU suite, then SSB with and without accept-mask leaves and the
# inverted sweep at expansion groups of 8 (default), 4 and 1 chunks.
set -o pipefail
bash scripts/gpu_tests.sh || exit 1
SWEEP="none PINOT_AMD_LEAF_MASKS=0" ARGS="--workload ssb" bash scripts/gpu_sweep.sh || exit 1
cp gpurun_out/sweep.txt gpurun_out/sweep_ssb_masks.txt
SWEEP="none PINOT_AMD_EXPAND_GROUP=4 PINOT_AMD_EXPAND_GROUP=1" ARGS="--workload inverted" bash scripts/gpu_sweep.sh || exit 1
cp gpurun_out/sweep.txt gpurun_out/sweep_inv_group.txt
