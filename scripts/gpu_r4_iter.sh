# One iteration of round-4 kernel work on a GPU box: the affected GPU tests, then the sweeps.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_widekeys.py tests/test_gpu_groupby_highcard.py tests/test_gpu_trim.py tests/test_gpu_packed_records.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_iter.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gputest_iter.log; exit 1; }
tail -2 gpurun_out/gputest_iter.log
SWEEP="${SWEEP_HC:-none PINOT_AMD_FLUSH_PAR=0}" ARGS="--workload highcard" STEPS=5 timeout -k 10 600 bash scripts/gpu_sweep.sh || exit 1
cp gpurun_out/sweep.txt gpurun_out/sweep_hc.txt
SWEEP="${SWEEP_WK:-none PINOT_AMD_HASH_LDS_SLOTS=2048}" ARGS="--workload wide-keys" STEPS=5 timeout -k 10 600 bash scripts/gpu_sweep.sh || exit 1
cp gpurun_out/sweep.txt gpurun_out/sweep_wk.txt
