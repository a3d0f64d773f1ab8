# LDS accept tables: the GPU suite, then SSB with and without them.
set -o pipefail
bash scripts/gpu_tests.sh || exit 1
SWEEP="none PINOT_AMD_LEAF_LUT=0" ARGS="--workload ssb" bash scripts/gpu_sweep.sh || exit 1
cp gpurun_out/sweep.txt gpurun_out/sweep_ssb_lut.txt
