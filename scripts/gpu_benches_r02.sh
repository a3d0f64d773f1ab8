# Workload benches (configs[2], [3], [4]): one JSON line per query; summary table on stdout.
set -o pipefail
mkdir -p gpurun_out
for w in ${BENCHES:-highcard ssb inverted}; do
  timeout -k 10 500 python bench.py --workload $w --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline > gpurun_out/${w}_bench.json 2> gpurun_out/${w}_bench.err || { echo "$w FAILED"; tail -20 gpurun_out/${w}_bench.err; exit 1; }
  python -c "
import json
for l in open('gpurun_out/${w}_bench.json'):
    d = json.loads(l); r = d['roofline']; c = d['config']
    print('$w', c['scan_kernel'], 'sel=%.5f' % c['selectivity'], 'ms=%.3f' % d['ms_per_step'], 'rows/s=%.3g' % d['value'],
          'B/row=%.3f' % r['bytes_per_row'], 'frac=%.3f' % r['frac'], 'cold_ms=%.0f' % d['cold_ms'])
"
done
