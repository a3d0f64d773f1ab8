# inverted-index selectivity sweep at gated pipeline depths 1..4 (one JSON line per selectivity)
set -o pipefail
mkdir -p gpurun_out
for d in ${DEPTHS:-1 2 3 4}; do
  PINOT_AMD_GATE_DEPTH=$d timeout -k 10 400 python bench.py --workload inverted --segments ${SEGS:-40} --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/gd$d.json 2> gpurun_out/gd$d.err || { tail -5 gpurun_out/gd$d.err; exit 1; }
  python -c "
import json
for l in open('gpurun_out/gd$d.json'):
    d = json.loads(l); r = d['roofline']
    print('depth $d', 'sel=%.5f' % d['config']['selectivity'], 'ms=%.3f' % d['ms_per_step'], 'kernel_ms=%.3f' % r['kernel_ms'], 'frac=%.3f' % r['frac'])
"
done
