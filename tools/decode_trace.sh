# Batch-N decode: wall time per step, then a rocprofv3 kernel trace of the same loop -> gpurun_out/trace_dec<N>/
set -o pipefail
R=$PWD
N=${1:-1}
O=$R/gpurun_out/trace_dec$N
mkdir -p $O
timeout -k 10 200 python3 $R/tools/decode_profile.py --batch $N --prompt 173 --new 128 > $O/wall.txt 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d /tmp/td$N -o run -- python3 $R/tools/decode_profile.py --batch $N --prompt 173 --new 128 > $O/log.txt 2>&1 || exit $?
find /tmp/td$N -name "*kernel_stats.csv" -exec cp {} $O/ \;
find /tmp/td$N -name "*kernel_trace.csv" -exec cp {} $O/ \;
rm -rf /tmp/td$N
