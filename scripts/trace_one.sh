# Kernel trace (rocprofv3 --kernel-trace --stats) of one bench workload; prints the per-kernel stats.
# ARGS: bench.py arguments (e.g. "--workload highcard --segments 40").
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/trace_one
rm -rf $D; mkdir -p $D
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $D/t -o run -- python3 bench.py $ARGS --no-cpu-baseline --steps ${STEPS:-10} --warmup 2 > $D/bench.json 2> $D/err.log || { tail -5 $D/err.log; exit 1; }
f=$(find $D/t -name "*kernel_stats.csv" | head -1)
cp "$f" $D/kernel_stats.csv
python3 -c "
import csv
for r in csv.DictReader(open('$D/kernel_stats.csv')):
    print('%-60s calls=%5s avg_ms=%.4f tot_pct=%s' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e6, r['Percentage']))
"
find $D/t -name "*kernel_trace.csv" | xargs rm -f
