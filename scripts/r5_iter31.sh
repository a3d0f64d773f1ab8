# Round 5, thirty-first GPU iteration: configs[3] at the default limit three times (run-to-run spread of the line
# after the scatter self-check: 6.29 ms before it, 6.49 ms in iteration 30).
set -o pipefail
mkdir -p gpurun_out/r5_iter31
for i in 1 2 3; do
  timeout -k 10 400 python bench.py --workload highcard-default --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r5_iter31/hcdef$i.json 2> gpurun_out/r5_iter31/hcdef$i.err || { echo "run $i FAILED"; tail -5 gpurun_out/r5_iter31/hcdef$i.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r5_iter31/hcdef$i.json').read().strip().splitlines()[-1]); print('hcdef run $i', round(d['ms_per_step'],3), 'ms/step kernel', round(d['roofline']['kernel_ms'],3))"
done
