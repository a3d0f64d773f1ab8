set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_groupby_highcard.py -x -v --timeout 120 --timeout-method thread > gpurun_out/hc_test.log 2>&1 || { echo HC_TEST_FAILED; tail -30 gpurun_out/hc_test.log; exit 1; }
tail -3 gpurun_out/hc_test.log
timeout -k 10 300 python bench.py --workload highcard --segments 20 --steps 5 --warmup 1 --no-cpu-baseline --check > gpurun_out/hc_bench_part.json 2> gpurun_out/hc_bench_part.err || { echo BENCH_FAILED; tail -20 gpurun_out/hc_bench_part.err; exit 1; }
cat gpurun_out/hc_bench_part.json
mkdir -p gpurun_out/prof_hc
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_hc/trace -o run -- python3 bench.py --workload highcard --segments 20 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_hc/bench.json 2> gpurun_out/prof_hc/bench.err
grep pinot gpurun_out/prof_hc/trace/run_kernel_stats.csv
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_hc/pmc2 -o run -- python3 bench.py --workload highcard --segments 20 --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> gpurun_out/prof_hc/pmc2.err
echo pmc2 done
