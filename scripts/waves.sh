set -o pipefail
mkdir -p gpurun_out
for w in 0 5 6 7; do
PINOT_AMD_WAVES_PER_EU=$w timeout -k 10 300 python bench.py --segments 40 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/w$w.json 2> gpurun_out/w$w.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/w$w.json')); print('waves $w', d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
for w in 0 6 8; do
PINOT_AMD_WAVES_PER_EU=$w timeout -k 10 300 python bench.py --workload ssb --query-index 0 --segments 20 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ws$w.json 2> gpurun_out/ws$w.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/ws$w.json')); print('ssb q1.1 waves $w', d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
