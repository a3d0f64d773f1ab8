set -o pipefail
mkdir -p gpurun_out
for qi in 0 3; do for n in 20 60 180; do
timeout -k 10 300 python bench.py --workload ssb --query-index $qi --segments $n --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/sc.json 2> gpurun_out/sc.err || { tail -5 gpurun_out/sc.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/sc.json')); print('q $qi segs $n', round(d['roofline']['kernel_ms'],4), round(d['roofline']['frac'],3))"
done; done
