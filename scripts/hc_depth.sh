set -o pipefail
mkdir -p gpurun_out
for d in 1 2 3; do
PINOT_AMD_PREFETCH=$d timeout -k 10 300 python bench.py --workload highcard --segments 20 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/hc_d$d.json 2> gpurun_out/hc_d$d.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/hc_d$d.json')); print('depth $d', d['roofline']['kernel_ms'])"
done
