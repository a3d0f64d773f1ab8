# Round 5, tenth GPU iteration: one-word LDS probes read together, the LDS-sorted spill scatter by default --
# hash-plan parity (wide keys, the parity sweep's hash mode, SSB through the hash plan), the wide-key line at
# 100 segments with its per-dispatch trace.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_widekeys.py tests/test_gpu_parity.py tests/test_gpu_ssb.py tests/test_gpu_filter_gate.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r5_gputest10.log 2>&1 || { echo GPU_TEST_FAILED; tail -60 gpurun_out/r5_gputest10.log; exit 1; }
tail -2 gpurun_out/r5_gputest10.log
D=gpurun_out/r5_trace_wk10
mkdir -p $D
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d $D -o run -- python3 bench.py --workload wide-keys --steps 5 --warmup 2 --no-cpu-baseline > $D/bench.json 2> $D/bench.err || { echo trace failed; tail -5 $D/bench.err; exit 1; }
python scripts/trace_tail.py $(find $D -name "run_kernel_trace.csv") 5 > $D/tail.txt
find $D -name "run_kernel_trace.csv" | xargs rm -f
head -5 $D/tail.txt
head -c 300 $D/bench.json
