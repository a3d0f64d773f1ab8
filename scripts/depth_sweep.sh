set -o pipefail
mkdir -p gpurun_out
for qi in 0 3 6 10; do for d in 2 3 4 6 8; do
PINOT_AMD_PREFETCH=$d timeout -k 10 300 python bench.py --workload ssb --query-index $qi --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/sd.json 2> gpurun_out/sd.err || { tail -5 gpurun_out/sd.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/sd.json')); print('q $qi depth $d', round(d['roofline']['kernel_ms'],4))"
done; done
for d in 1 2 3 4; do
PINOT_AMD_PREFETCH=$d timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/sd.json 2> gpurun_out/sd.err || { tail -5 gpurun_out/sd.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/sd.json')); print('scan depth $d', round(d['roofline']['kernel_ms'],4))"
done
