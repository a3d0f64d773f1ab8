set -e
mkdir -p gpurun_out/prof
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace -o run -- python3 bench.py --steps 10 --warmup 2 --segments 40 --no-cpu-baseline > gpurun_out/prof/trace_bench.json 2> gpurun_out/prof/trace_bench.err
echo trace done
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/pmc1 -o run -- python3 bench.py --steps 3 --warmup 1 --segments 40 --no-cpu-baseline > /dev/null 2> gpurun_out/prof/pmc1.err
echo pmc1 done
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES --output-format csv -d gpurun_out/prof/pmc2 -o run -- python3 bench.py --steps 3 --warmup 1 --segments 40 --no-cpu-baseline > /dev/null 2> gpurun_out/prof/pmc2.err
echo pmc2 done
