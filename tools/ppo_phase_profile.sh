set -o pipefail
R=$PWD
mkdir -p $R/gpurun_out/prof_ppo
cd /tmp && export TMPDIR=/tmp
timeout -k 10 700 rocprofv3 --kernel-trace --marker-trace --stats -f csv -d /tmp/pp -o run -- python3 $R/bench.py --steps 1 --warmup 1 > $R/gpurun_out/prof_ppo/log.txt 2>&1 || exit $?
python3 $R/tools/phase_breakdown.py /tmp/pp --top 25 --grids "${GRIDS:-gemm_tile_kernel,gemm_256_kernel}" > $R/gpurun_out/prof_ppo/phases.txt 2>&1
find /tmp/pp -name "*kernel_stats.csv" -exec cp {} $R/gpurun_out/prof_ppo/ \;
rm -rf /tmp/pp
