# rocprofv3 recipe for the round-1 profiles (run on the GPU box from the repo root):
#   bash profiles/profile_r01.sh
# Kernel trace + stats of the default bench (configs[1], 40 segments = 400M rows to keep the PMC
# passes short) and of the other workloads, then separate PMC passes for the hot kernel (FETCH_SIZE;
# WRITE_SIZE; SQ counters), then profiles/summarize.py writes the JSON summaries.
set -e
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
ARGS="--steps 10 --warmup 2 --segments 40 --no-cpu-baseline"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace -o run -- python3 bench.py $ARGS > gpurun_out/prof/trace_bench.json 2> gpurun_out/prof/trace_bench.err
echo trace done
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace_hc -o run -- python3 bench.py --workload highcard --steps 5 --warmup 1 --segments 40 --no-cpu-baseline > gpurun_out/prof/trace_hc.json 2> gpurun_out/prof/trace_hc.err
echo trace_hc done
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace_ssb -o run -- python3 bench.py --workload ssb --steps 5 --warmup 1 --segments 20 --no-cpu-baseline > gpurun_out/prof/trace_ssb.json 2> gpurun_out/prof/trace_ssb.err
echo trace_ssb done
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/pmc1 -o run -- python3 bench.py --steps 3 --warmup 1 --segments 40 --no-cpu-baseline > /dev/null 2> gpurun_out/prof/pmc1.err
echo pmc1 done
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof/pmc3 -o run -- python3 bench.py --steps 3 --warmup 1 --segments 40 --no-cpu-baseline > /dev/null 2> gpurun_out/prof/pmc3.err
echo pmc3 done
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES --output-format csv -d gpurun_out/prof/pmc2 -o run -- python3 bench.py --steps 3 --warmup 1 --segments 40 --no-cpu-baseline > /dev/null 2> gpurun_out/prof/pmc2.err
echo pmc2 done
python3 profiles/summarize.py gpurun_out/prof gpurun_out/prof_summary
