# One GPU iteration: the GPU tests named in $TESTS (default: the whole -m gpu suite), then one bench
# line per workload in $BENCHES (default: "default"; e.g. "default highcard ssb inverted"), each step
# under its own time limit, stopping at the first failure.
set -o pipefail
mkdir -p gpurun_out
if [ "${TESTS:-}" != "none" ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1 || { echo GPU_TEST_FAILED; grep -E "^(FAILED|ERROR)|^E " gpurun_out/gputest.log | head -40; tail -3 gpurun_out/gputest.log; exit 1; }
  tail -2 gpurun_out/gputest.log
fi
for w in ${BENCHES:-default}; do
  case $w in
    default) A="" ;;
    *) A="--workload $w" ;;
  esac
  timeout -k 10 500 python bench.py $A --no-cpu-baseline --steps ${STEPS:-10} ${BENCH_ARGS:-} > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err || { echo BENCH_FAILED $w; tail -20 gpurun_out/bench_$w.err; exit 1; }
  python -c "
import json
for l in open('gpurun_out/bench_$w.json'):
    d = json.loads(l); r = d['roofline']; c = d['config']
    print('$w', c.get('scan_kernel'), '%.4f' % c.get('selectivity', 0), 'ms=%.3f' % d['ms_per_step'], 'value=%.3e' % d['value'], 'kernel_ms=%.3f' % r.get('kernel_ms', 0), 'B/row=%.2f' % r.get('bytes_per_row', 0), 'frac=%.3f' % r['frac'], 'cold_ms=%s' % d.get('cold_ms'))
"
done
