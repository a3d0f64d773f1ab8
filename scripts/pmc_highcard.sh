set -o pipefail
mkdir -p gpurun_out/prof_hc
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES --output-format csv -d gpurun_out/prof_hc/pmc3 -o run -- python3 bench.py --workload highcard --segments 20 --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> gpurun_out/prof_hc/pmc3.err
echo pmc3 done
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_hc/pmc1 -o run -- python3 bench.py --workload highcard --segments 20 --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> gpurun_out/prof_hc/pmc1.err
echo pmc1 done
