# Round 5, eleventh GPU iteration: LDS-typed hash probes (no flat loads / vmcnt(0) per probe), global-typed
# roaring expansion loads -- hash / inverted / spill parity, then the wide-key and inverted lines.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_widekeys.py tests/test_gpu_inverted.py tests/test_gpu_parity.py tests/test_gpu_ssb.py tests/test_gpu_trim.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r5_gputest11.log 2>&1 || { echo GPU_TEST_FAILED; tail -60 gpurun_out/r5_gputest11.log; exit 1; }
tail -2 gpurun_out/r5_gputest11.log
D=gpurun_out/r5_trace_wk11
mkdir -p $D
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d $D -o run -- python3 bench.py --workload wide-keys --steps 5 --warmup 2 --no-cpu-baseline > $D/bench.json 2> $D/bench.err || { echo trace failed; tail -5 $D/bench.err; exit 1; }
python scripts/trace_tail.py $(find $D -name "run_kernel_trace.csv") 5 > $D/tail.txt
find $D -name "run_kernel_trace.csv" | xargs rm -f
head -5 $D/tail.txt
head -c 300 $D/bench.json; echo
timeout -k 10 300 python bench.py --workload inverted --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r5_inv11.json 2> gpurun_out/r5_inv11.err || { echo inverted FAILED; tail -5 gpurun_out/r5_inv11.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/r5_inv11.json'):
    d = json.loads(l); print(d['config']['selectivity'], d['config']['scan_kernel'], round(d['ms_per_step'], 4))
"
