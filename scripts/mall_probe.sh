set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/mall
for n in 1 4 40; do
  timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/mall/s$n -o run -- python3 bench.py --workload highcard --segments $n --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/mall/s$n.json 2> gpurun_out/mall/s$n.err || { echo "s$n failed"; tail -5 gpurun_out/mall/s$n.err; exit 1; }
  grep -h "pinot_part" gpurun_out/mall/s$n/run_kernel_stats.csv | cut -d, -f1-4
  rm -f gpurun_out/mall/s$n/run_kernel_trace.csv
done
