# configs[3] (20 segments): scatter flush threshold sweep (percent of the staging capacity)
set -o pipefail
mkdir -p gpurun_out
for f in ${PCTS:-35 50 65 80}; do
PINOT_AMD_FLUSH_PCT=$f timeout -k 10 300 python bench.py --workload highcard --segments 20 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/hc_f$f.json 2> gpurun_out/hc_f$f.err || { tail -5 gpurun_out/hc_f$f.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/hc_f$f.json')); print('flush pct $f', round(d['roofline']['kernel_ms'], 3))"
done
