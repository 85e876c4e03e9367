# Kernel statistics of the batch-N decode loop (tools/decode_profile.py) -> gpurun_out/prof_dec<N>/
set -o pipefail
R=$PWD
N=${1:-256}
mkdir -p $R/gpurun_out/prof_dec$N
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d /tmp/pd$N -o run -- python3 $R/tools/decode_profile.py --batch $N --prompt 173 --new 128 > $R/gpurun_out/prof_dec$N/log.txt 2>&1 || exit $?
find /tmp/pd$N -name "*kernel_stats.csv" -exec cp {} $R/gpurun_out/prof_dec$N/ \;
rm -rf /tmp/pd$N
