# Round 5, fourteenth GPU iteration: LDS admission by recurrence on by default (2^-5), spill regions grown from
# what an overflowing execution needed -- hash-plan parity, the admission sweep at 100 segments, the line.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_widekeys.py tests/test_gpu_parity.py tests/test_gpu_ssb.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r5_gputest14.log 2>&1 || { echo GPU_TEST_FAILED; tail -60 gpurun_out/r5_gputest14.log; exit 1; }
tail -2 gpurun_out/r5_gputest14.log
SWEEP="none PINOT_AMD_HASH_LDS_ADMIT=4 PINOT_AMD_HASH_LDS_ADMIT=6 PINOT_AMD_HASH_LDS_ADMIT=7 PINOT_AMD_HASH_LDS_ADMIT=0" ARGS="--workload wide-keys" STEPS=5 timeout -k 10 900 bash scripts/gpu_sweep.sh || exit 1
cp gpurun_out/sweep.txt gpurun_out/r5_sweep_wk_admit.txt
D=gpurun_out/r5_trace_wk14
mkdir -p $D
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d $D -o run -- python3 bench.py --workload wide-keys --steps 5 --warmup 2 --no-cpu-baseline > $D/bench.json 2> $D/bench.err || { echo trace failed; tail -5 $D/bench.err; exit 1; }
python scripts/trace_tail.py $(find $D -name "run_kernel_trace.csv") 5 > $D/tail.txt
find $D -name "run_kernel_trace.csv" | xargs rm -f
head -5 $D/tail.txt
