# Round 5, thirteenth GPU iteration: why the wide-key scan takes 2.3x longer per row at 100 segments than at 40 --
# spill-region capacity (records past it take the HBM table) and LDS admission by recurrence, at 100 segments.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_widekeys.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r5_gputest13.log 2>&1 || { echo GPU_TEST_FAILED; tail -60 gpurun_out/r5_gputest13.log; exit 1; }
tail -2 gpurun_out/r5_gputest13.log
SWEEP="none PINOT_AMD_SPILL_BYTES=25769803776 PINOT_AMD_HASH_LDS_ADMIT=3 PINOT_AMD_HASH_LDS_ADMIT=3,PINOT_AMD_SPILL_BYTES=25769803776 PINOT_AMD_HASH_LDS_ADMIT=5,PINOT_AMD_SPILL_BYTES=25769803776" ARGS="--workload wide-keys" STEPS=5 timeout -k 10 900 bash scripts/gpu_sweep.sh || exit 1
cp gpurun_out/sweep.txt gpurun_out/r5_sweep_wk_cap.txt
