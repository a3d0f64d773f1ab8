# Round 5, fourth GPU iteration: the hash plan's second level (LDS misses spilled and aggregated per key-hash
# partition): hash-plan parity, the wide-key line with / without it; scatter knobs on the default-limit configs[3].
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_widekeys.py tests/test_gpu_server_trim.py tests/test_gpu_dist.py "tests/test_gpu_parity.py" -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r5_gputest4.log 2>&1 || { echo GPU_TEST_FAILED; tail -60 gpurun_out/r5_gputest4.log; exit 1; }
tail -2 gpurun_out/r5_gputest4.log
SWEEP="none PINOT_AMD_HASH_SPILL=0" ARGS="--workload wide-keys --segments 40" STEPS=5 timeout -k 10 400 bash scripts/gpu_sweep.sh || exit 1
cp gpurun_out/sweep.txt gpurun_out/r5_sweep_widekeys_spill.txt
SWEEP="none PINOT_AMD_FLUSH_EVERY=4 PINOT_AMD_PREFETCH=2 PINOT_AMD_NT_LOADS=1 PINOT_AMD_FLUSH_EVERY=4,PINOT_AMD_PREFETCH=2" ARGS="--workload highcard-default --segments 40" STEPS=10 timeout -k 10 400 bash scripts/gpu_sweep.sh || exit 1
cp gpurun_out/sweep.txt gpurun_out/r5_sweep_hcdef_knobs.txt
SWEEP="none PINOT_AMD_FLUSH_EVERY=2 PINOT_AMD_NT_LOADS=1" ARGS="--workload highcard --segments 40" STEPS=10 timeout -k 10 400 bash scripts/gpu_sweep.sh || exit 1
cp gpurun_out/sweep.txt gpurun_out/r5_sweep_hc_knobs.txt
