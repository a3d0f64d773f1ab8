# Round 5, eighth GPU iteration: filter-gated fused scans -- parity (forced gate over the random sweep, ragged
# segments, SSB golden; the planner's choice on SSB), SSB timing with the planner's choice vs the gate off; then
# the counters of iteration 7 (wide-key kernels, Q4.2 select pass, configs[3] scatter).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_filter_gate.py tests/test_gpu_ssb.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r5_gputest8.log 2>&1 || { echo GPU_TEST_FAILED; tail -60 gpurun_out/r5_gputest8.log; exit 1; }
tail -2 gpurun_out/r5_gputest8.log
SWEEP="none PINOT_AMD_FILTER_GATE=0 PINOT_AMD_FILTER_GATE=1,PINOT_AMD_SELECT=never" ARGS="--workload ssb" STEPS=10 timeout -k 10 600 bash scripts/gpu_sweep.sh || exit 1
cp gpurun_out/sweep.txt gpurun_out/r5_sweep_ssb_fgate.txt
bash scripts/r5_iter7.sh
