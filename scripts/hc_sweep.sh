# configs[3] knob sweep (20 segments): prefetch depth x staging capacity; one JSON line per point
set -o pipefail
mkdir -p gpurun_out
for d in ${DEPTHS:-1 2 3}; do
for c in ${CAPS:-40}; do
PINOT_AMD_PREFETCH=$d PINOT_AMD_STAGE_CAP=$c timeout -k 10 300 python bench.py --workload highcard --segments 20 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/hc_d${d}_c$c.json 2> gpurun_out/hc_d${d}_c$c.err || { tail -5 gpurun_out/hc_d${d}_c$c.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/hc_d${d}_c$c.json')); print('depth $d cap $c', round(d['roofline']['kernel_ms'], 3))"
done
done
