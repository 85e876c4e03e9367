set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/r6/dp_direct_debug.py > gpurun_out/dp_debug.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/dp_debug.log | tail -20; exit $rc
