# inverted sweep point (QI, default the 1 % query) with the forward index forced (PINOT_AMD_INV_POLICY=never)
set -o pipefail
mkdir -p gpurun_out
PINOT_AMD_INV_POLICY=never timeout -k 10 300 python bench.py --workload inverted --no-cpu-baseline --steps 5 --query-index ${QI:-2} > gpurun_out/inv_never.json 2> gpurun_out/inv_never.err || { tail -5 gpurun_out/inv_never.err; exit 1; }
python -c "
import json
d = json.loads(open('gpurun_out/inv_never.json').readlines()[-1])
print('inv never', d['config']['selectivity'], d['config']['scan_kernel'], round(d['ms_per_step'], 3))
"
