mkdir -p gpurun_out/r3 && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "fp8_decode_w8a16 or swiglu_pair" > gpurun_out/r3/test_fp8_5.log 2>&1 || { echo "tests failed"; exit 1; }
timeout -k 10 300 python -u tools/fp8_decode_table.py --ms 1,16,24,32,48,64 --splits 1,2,4,8,16 > gpurun_out/r3/fp8_decode_table_5.log 2>&1 || { echo "table failed"; exit 1; }
timeout -k 10 450 python -u bench.py --mode pipeline --steps 2 --warmup 1 > gpurun_out/r3/bench_pipeline_fp8_5.log 2>&1
