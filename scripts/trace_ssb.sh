set -o pipefail
mkdir -p gpurun_out/trace_ssb
export TMPDIR=/tmp
W=/tmp/trwork
for qi in ${QIS:-0 3}; do
rm -rf $W
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $W -o run -- python3 bench.py --workload ssb --query-index $qi --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/trace_ssb/bench_q$qi.json 2> gpurun_out/trace_ssb/q$qi.err || exit 1
f=$(find $W -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/trace_ssb/stats_q$qi.csv
f=$(find $W -name "*kernel_trace.csv" | head -1); { head -1 "$f"; grep -E "pinot|init_acc" "$f" | tail -40 || true; } > gpurun_out/trace_ssb/trace_q$qi.csv
done
echo done
