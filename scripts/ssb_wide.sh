set -o pipefail
mkdir -p gpurun_out
run() {  # qi label env...
  qi=$1; lab=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --workload ssb --query-index $qi --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/sw.json 2> gpurun_out/sw.err || { tail -5 gpurun_out/sw.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/sw.json')); print('q $qi $lab', round(d['roofline']['kernel_ms'],4), d['config']['scan_kernel'])"
}
for qi in 3 6 11; do
  run $qi default X=1
  run $qi nowide PINOT_AMD_WIDE_LDS=0
  run $qi nowide_noatomic PINOT_AMD_WIDE_LDS=0 PINOT_AMD_SAMPLE_STRIDE=0 PINOT_AMD_ATOMIC_HANDOVER=0
  run $qi depth4 PINOT_AMD_PREFETCH=4
  run $qi depth1 PINOT_AMD_PREFETCH=1
done
