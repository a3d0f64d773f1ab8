# Select-path parity (select tests, SSB / inverted parity) then the SSB and inverted sweeps.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_select.py tests/test_gpu_parity.py -m gpu > gpurun_out/gputest_sel.log 2>&1 || { echo GPU_TEST_FAILED; tail -60 gpurun_out/gputest_sel.log; exit 1; }
tail -2 gpurun_out/gputest_sel.log
SWEEP="none" ARGS="--workload ssb" bash scripts/gpu_sweep.sh || exit 1
cp gpurun_out/sweep.txt gpurun_out/sweep_ssb_runs.txt
SWEEP="none PINOT_AMD_EXPAND_GROUP=2" ARGS="--workload inverted" bash scripts/gpu_sweep.sh || exit 1
cp gpurun_out/sweep.txt gpurun_out/sweep_inv_runs.txt
