set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/r5c1
timeout -k 10 200 tools/gemm_exp/bin/gemm_exp_base 10 - 0,240,228,208,192,160,128 > gpurun_out/r5c1/cu_mask.log 2>&1 || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5c1/libprof -o lib -- python3 tools/gemm_big_probe.py --cases lib_nt,nt,lib_nn,nn --shapes qkv,gate_up,o,down --rounds 2 > gpurun_out/r5c1/libprobe.log 2>&1 || exit 2
timeout -k 10 400 python3 bench.py --steps 5 --warmup 2 > gpurun_out/r5c1/bench.log 2>&1 || exit 3
