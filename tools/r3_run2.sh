mkdir -p gpurun_out/r3 && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "fp8 or swiglu_pair" > gpurun_out/r3/test_fp8_2.log 2>&1 || { echo "fp8 tests failed"; exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_pipeline_gpu.py -x -v --timeout 240 --timeout-method thread -k "early_exit or checkpointing or config5" > gpurun_out/r3/test_pipeline_new.log 2>&1 || { echo "pipeline tests failed"; exit 1; }
timeout -k 10 400 python -u tools/fp8_decode_table.py --ms 1,4,16,24,32,48,64 --splits 1,2,4,8 > gpurun_out/r3/fp8_decode_table_2.log 2>&1 || { echo "table failed"; exit 1; }
timeout -k 10 450 python -u bench.py --mode pipeline --steps 2 --warmup 1 > gpurun_out/r3/bench_pipeline_fp8_2.log 2>&1
