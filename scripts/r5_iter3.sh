# Round 5, third GPU iteration: the default-limit configs[3] scatter with the segment's admission bitmap in
# LDS: parity (trim + full-size tests), A/B timing at 40 segments, and a kernel trace at the bench's 100 segments.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_trim.py tests/test_gpu_groupby_highcard.py tests/test_gpu_server_trim.py "tests/test_gpu_fullsize.py::test_full_size_highcard_default_limit_vs_oracle" -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r5_gputest3.log 2>&1 || { echo GPU_TEST_FAILED; tail -60 gpurun_out/r5_gputest3.log; exit 1; }
tail -2 gpurun_out/r5_gputest3.log
SWEEP="none PINOT_AMD_ADMIT_LDS=0" ARGS="--workload highcard-default --segments 40" STEPS=10 timeout -k 10 300 bash scripts/gpu_sweep.sh || exit 1
cp gpurun_out/sweep.txt gpurun_out/r5_sweep_hcdef_lds.txt
D=gpurun_out/r5_trace_hcdef100
mkdir -p $D
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 bench.py --workload highcard-default --steps 10 --warmup 2 --no-cpu-baseline > $D/bench.json 2> $D/bench.err || { echo trace failed; tail -5 $D/bench.err; exit 1; }
find $D -name "run_kernel_trace.csv" | xargs rm -f
head -c 600 $D/bench.json
