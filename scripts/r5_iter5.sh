# Round 5, fifth GPU iteration: the device block pool (cached host planning) -- parity of the paths that
# allocate most per plan, the cached-plan latency of configs[1] / SSB / inverted, and a kernel trace of the
# wide-key hash plan with its spill level at the bench's 100 segments.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_inverted.py tests/test_gpu_select.py tests/test_gpu_empty_segments.py tests/test_gpu_pinot_written.py tests/test_gpu_bench_ranks.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r5_gputest5.log 2>&1 || { echo GPU_TEST_FAILED; tail -60 gpurun_out/r5_gputest5.log; exit 1; }
tail -2 gpurun_out/r5_gputest5.log
D=gpurun_out/r5_plan
mkdir -p $D
for w in scan ssb inverted; do
  timeout -k 10 300 python bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline > $D/$w.json 2> $D/$w.err || { echo "$w FAILED"; tail -5 $D/$w.err; exit 1; }
done
python scripts/plan_summary.py $D/*.json | tee $D/summary.txt
D=gpurun_out/r5_trace_wk100
mkdir -p $D
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 bench.py --workload wide-keys --steps 5 --warmup 2 --no-cpu-baseline > $D/bench.json 2> $D/bench.err || { echo trace failed; tail -5 $D/bench.err; exit 1; }
find $D -name "run_kernel_trace.csv" | xargs rm -f
head -c 400 $D/bench.json
