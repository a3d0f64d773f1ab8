set -o pipefail
mkdir -p gpurun_out/prof_hc
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_hc/trace -o run -- python3 bench.py --workload highcard --segments 20 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_hc/bench.json 2> gpurun_out/prof_hc/bench.err
echo trace done
find gpurun_out/prof_hc -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-200
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_hc/pmc1 -o run -- python3 bench.py --workload highcard --segments 20 --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> gpurun_out/prof_hc/pmc1.err
echo pmc1 done
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_hc/pmc2 -o run -- python3 bench.py --workload highcard --segments 20 --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> gpurun_out/prof_hc/pmc2.err
echo pmc2 done
