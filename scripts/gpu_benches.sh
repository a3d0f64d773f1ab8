# Every BASELINE workload's bench lines (one JSON line per query) with the CPU baseline, on a GPU box:
#   BENCHES="scan highcard highcard-default inverted ssb" bash scripts/gpu_benches.sh
# Lines land in gpurun_out/<workload>_bench.json; a summary table goes to stdout.
set -o pipefail
mkdir -p gpurun_out
for w in ${BENCHES:-scan highcard inverted ssb highcard-default}; do
  timeout -k 10 ${BENCH_TIMEOUT:-420} python bench.py --workload $w --steps ${STEPS:-10} --warmup 2 ${BENCH_ARGS:-} > gpurun_out/${w}_bench.json 2> gpurun_out/${w}_bench.err || { echo "$w FAILED"; tail -20 gpurun_out/${w}_bench.err; exit 1; }
  python -c "
import json
for l in open('gpurun_out/${w}_bench.json'):
    d = json.loads(l); r = d['roofline']; c = d['config']; cpu = d.get('cpu_baseline') or {}
    print('$w', c['scan_kernel'], 'sel=%.5f' % c['selectivity'], 'ms=%.3f' % d['ms_per_step'], 'kernel_ms=%.3f' % r['kernel_ms'],
          'rows/s=%.3g' % d['value'], 'B/row=%.3f' % r['bytes_per_row'], 'frac=%.3f' % r['frac'], 'cold_ms=%.0f' % d['cold_ms'],
          'plan_ms=%.1f' % d['cached_plan_ms'], 'cpu=%.3g' % cpu.get('value', 0))
"
done
