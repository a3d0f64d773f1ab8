# Round 5, second GPU iteration: the full GPU suite on the new host paths (segment-level trim, remembered hash
# capacities, device sort of hash groups, bitset slack), a kernel trace of the default-limit configs[3] plan with
# XCD-aware ranges, the wide-key line (re-issued query latency), and XCD remap A/B on other plans.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r5_gputest2.log 2>&1 || { echo GPU_TEST_FAILED; tail -60 gpurun_out/r5_gputest2.log; exit 1; }
tail -2 gpurun_out/r5_gputest2.log
D=gpurun_out/r5_trace_hcdef
mkdir -p $D
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 bench.py --workload highcard-default --segments 40 --steps 10 --warmup 2 --no-cpu-baseline > $D/bench.json 2> $D/bench.err || { echo trace failed; tail -5 $D/bench.err; exit 1; }
find $D -name "run_kernel_trace.csv" | xargs rm -f
timeout -k 10 300 python bench.py --workload wide-keys --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r5_widekeys.json 2> gpurun_out/r5_widekeys.err || { echo WK_FAILED; tail -5 gpurun_out/r5_widekeys.err; exit 1; }
cat gpurun_out/r5_widekeys.json
SWEEP="none PINOT_AMD_XCD_REMAP=1" ARGS="--segments 100" STEPS=10 timeout -k 10 300 bash scripts/gpu_sweep.sh || exit 1
cp gpurun_out/sweep.txt gpurun_out/r5_sweep_scan_xcd.txt
: > gpurun_out/r5_sweep_ssb_xcd.txt
for q in 3 6 11; do
  SWEEP="none PINOT_AMD_XCD_REMAP=1" ARGS="--workload ssb --query-index $q" STEPS=10 timeout -k 10 300 bash scripts/gpu_sweep.sh || exit 1
  cat gpurun_out/sweep.txt >> gpurun_out/r5_sweep_ssb_xcd.txt
done
