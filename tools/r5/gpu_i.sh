#!/bin/bash
# round 5, GPU call I: clock and LDS instruction counts of gemm_big vs hipBLASLt on the update
# shapes (PMC per dispatch + kernel trace durations): cycles per GEMM vs effective clock
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
cd /tmp && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5i
mkdir -p $O
timeout -s KILL 300 rocprofv3 --pmc GRBM_COUNT SQ_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_BUSY_CU_CYCLES --kernel-trace --output-format csv -d $O/pmc -o p -- python3 $GRAFT_REPO_ROOT/tools/gemm_big_probe.py --M 9632 --cases nt,lib_nt --rounds 2 --iters 4 > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 1; }
tail -5 $O/run.log
