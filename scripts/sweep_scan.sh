# configs[1] scan kernel: pipeline depth x occupancy target x narrow sums (kernel ms per 1B rows)
set -o pipefail
mkdir -p gpurun_out
for cfg in "1 0 1" "2 0 1" "1 6 1" "1 8 1" "2 8 1" "1 0 0"; do
set -- $cfg
PINOT_AMD_PREFETCH=$1 PINOT_AMD_WAVES_PER_EU=$2 PINOT_AMD_NARROW_SUMS=$3 timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/sw.json 2> gpurun_out/sw.err || { tail -5 gpurun_out/sw.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/sw.json')); print('depth $1 waves $2 narrow $3', round(d['roofline']['kernel_ms'],4), round(d['roofline']['frac'],4))"
done
