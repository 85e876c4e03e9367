mkdir -p gpurun_out/r3 && export TMPDIR=/tmp
timeout -k 10 300 python -u tools/fp8_decode_table.py --ms 24,48,64 --splits 1,2,4,8 > gpurun_out/r3/fp8_decode_table_4.log 2>&1 || { echo "table failed"; exit 1; }
timeout -k 10 500 python -u bench.py --steps 0 --latency-contexts 1024,2048,4096 > gpurun_out/r3/bench_longctx.log 2>&1 || { echo "longctx failed"; exit 1; }
timeout -k 10 650 bash tools/prof_pipeline13b.sh > gpurun_out/r3/prof13b.log 2>&1 || { echo "prof13b failed"; exit 1; }
