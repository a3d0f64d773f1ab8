# Round 5, sixth GPU iteration: select-pass pipeline depth on SSB (bytes in flight per wave), and the
# untrimmed configs[3] scatter with its record stores wrapped into a cache-resident window (diagnostic: does
# the record round trip through HBM bound the scatter?), kernel traces of both cases; the wide-key plan's
# kernels per dispatch; the predicate leaf cache (parity, inverted cached plan).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_inverted.py tests/test_gpu_ssb.py tests/test_gpu_parity.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r5_gputest6.log 2>&1 || { echo GPU_TEST_FAILED; tail -60 gpurun_out/r5_gputest6.log; exit 1; }
tail -2 gpurun_out/r5_gputest6.log
mkdir -p gpurun_out/r5_plan6
timeout -k 10 300 python bench.py --workload inverted --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r5_plan6/inverted.json 2> gpurun_out/r5_plan6/inverted.err || { echo inverted FAILED; tail -5 gpurun_out/r5_plan6/inverted.err; exit 1; }
python scripts/plan_summary.py gpurun_out/r5_plan6/inverted.json
D=gpurun_out/r5_trace_wk100b
mkdir -p $D
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d $D -o run -- python3 bench.py --workload wide-keys --steps 5 --warmup 2 --no-cpu-baseline > $D/bench.json 2> $D/bench.err || { echo trace failed; tail -5 $D/bench.err; exit 1; }
python scripts/trace_tail.py $(find $D -name "run_kernel_trace.csv") 5 > $D/tail.txt
find $D -name "run_kernel_trace.csv" | xargs rm -f
head -12 $D/tail.txt
SWEEP="none PINOT_AMD_PREFETCH=2 PINOT_AMD_PREFETCH=3 PINOT_AMD_PREFETCH=4 PINOT_AMD_SEL_GROUP=2,PINOT_AMD_PREFETCH=3" ARGS="--workload ssb" STEPS=10 timeout -k 10 600 bash scripts/gpu_sweep.sh || exit 1
cp gpurun_out/sweep.txt gpurun_out/r5_sweep_ssb_depth.txt
for c in base wrap; do
  D=gpurun_out/r5_trace_hc_$c
  mkdir -p $D
  if [ $c = wrap ]; then export PINOT_AMD_DIAG_REC_WRAP=4194304; fi
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 bench.py --workload highcard --segments 40 --steps 10 --warmup 2 --no-cpu-baseline > $D/bench.json 2> $D/bench.err || { echo trace $c failed; tail -5 $D/bench.err; exit 1; }
  python scripts/trace_tail.py $(find $D -name "run_kernel_trace.csv") 10 > $D/tail.txt
  find $D -name "run_kernel_trace.csv" | xargs rm -f
  head -c 300 $D/bench.json; head -8 $D/tail.txt
done
