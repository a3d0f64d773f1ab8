# Round 5, ninth GPU iteration: filter-gated scans with unconditional (redirected) loads -- parity and SSB timing;
# the bitset-padding test; the wide-key spill scatter, per-lane record stores vs the LDS-sorted variant
# (per-dispatch trace at 100 segments, HBM write bytes at 40).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_filter_gate.py tests/test_gpu_ssb.py tests/test_gpu_inverted.py tests/test_gpu_widekeys.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r5_gputest9.log 2>&1 || { echo GPU_TEST_FAILED; tail -60 gpurun_out/r5_gputest9.log; exit 1; }
tail -2 gpurun_out/r5_gputest9.log
SWEEP="none PINOT_AMD_FILTER_GATE=0 PINOT_AMD_FILTER_GATE=1,PINOT_AMD_SELECT=never" ARGS="--workload ssb" STEPS=10 timeout -k 10 600 bash scripts/gpu_sweep.sh || exit 1
cp gpurun_out/sweep.txt gpurun_out/r5_sweep_ssb_fgate2.txt
for c in 0 1; do
  D=gpurun_out/r5_trace_wk_sort$c
  mkdir -p $D
  export PINOT_AMD_SPILL_SORT=$c
  timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d $D -o run -- python3 bench.py --workload wide-keys --steps 5 --warmup 2 --no-cpu-baseline > $D/bench.json 2> $D/bench.err || { echo trace $c failed; tail -5 $D/bench.err; exit 1; }
  python scripts/trace_tail.py $(find $D -name "run_kernel_trace.csv") 5 > $D/tail.txt
  find $D -name "run_kernel_trace.csv" | xargs rm -f
  head -4 $D/tail.txt
done
unset PINOT_AMD_SPILL_SORT
CASES="sort0|PINOT_AMD_SPILL_SORT=0|--workload wide-keys --segments 40;sort1|PINOT_AMD_SPILL_SORT=1|--workload wide-keys --segments 40" SETS="WRITE_SIZE;FETCH_SIZE" timeout -k 10 600 bash scripts/pmc_ab.sh > gpurun_out/r5_pmc_wk_sort.txt 2>&1 || { echo PMC_FAILED; tail -5 gpurun_out/r5_pmc_wk_sort.txt; exit 1; }
grep -A4 "spill_scatter" gpurun_out/r5_pmc_wk_sort.txt | head -20
