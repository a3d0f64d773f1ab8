# Round 5, thirtieth GPU iteration: configs[3] bench lines (untrimmed, default limit) with the scatter self-check.
set -o pipefail
mkdir -p gpurun_out/r5_iter30
for w in highcard highcard-default; do
  timeout -k 10 400 python bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r5_iter30/$w.json 2> gpurun_out/r5_iter30/$w.err || { echo "$w FAILED"; tail -5 gpurun_out/r5_iter30/$w.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/r5_iter30/$w.json').read().strip().splitlines()[-1]); print('$w', round(d['ms_per_step'],3), 'ms/step', d['roofline']['frac'])"
done
