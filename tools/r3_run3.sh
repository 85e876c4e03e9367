mkdir -p gpurun_out/r3 && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "fp8 or swiglu_pair or decode_step_fused" > gpurun_out/r3/test_fp8_3.log 2>&1 || { echo "tests failed"; exit 1; }
timeout -k 10 400 python -u tools/fp8_decode_table.py --ms 1,16,24,32,64 --splits 1,2,4,8 > gpurun_out/r3/fp8_decode_table_3.log 2>&1 || { echo "table failed"; exit 1; }
