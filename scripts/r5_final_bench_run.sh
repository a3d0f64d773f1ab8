COMMIT=dff77ab bash scripts/r5_final_bench.sh
