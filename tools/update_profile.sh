set -o pipefail
R=$PWD
mkdir -p $R/gpurun_out/prof_upd
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d /tmp/pu -o run -- python3 $R/tools/update_probe.py --iters 1 > $R/gpurun_out/prof_upd/log.txt 2>&1 || exit $?
find /tmp/pu -name "*.csv" -exec cp {} $R/gpurun_out/prof_upd/ \;
rm -rf /tmp/pu
