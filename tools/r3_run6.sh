mkdir -p gpurun_out/r3 && export TMPDIR=/tmp
timeout -k 10 300 python -u tools/fp8_decode_table.py --ms 1,2,4,8,16,24,32,48,64 > gpurun_out/r3/fp8_decode_table_6.log 2>&1 || { echo "table failed"; exit 1; }
timeout -k 10 650 bash tools/prof_pipeline13b.sh > gpurun_out/r3/prof13b_2.log 2>&1 || { echo "prof13b failed"; exit 1; }
timeout -k 10 300 bash tools/fetch_size_calibration.sh > gpurun_out/r3/fetch_cal.log 2>&1 || { echo "fetch cal failed"; exit 1; }
timeout -k 10 400 bash tools/gemm_ab_pmc.sh > gpurun_out/r3/gemm_ab.log 2>&1 || { echo "gemm ab failed"; exit 1; }
