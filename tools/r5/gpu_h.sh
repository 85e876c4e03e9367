#!/bin/bash
# round 5, GPU call H: effective shader clock of the large GEMMs (PMC cycle counters per dispatch
# against the kernel trace's duration): is the 256x256 GEMM running below the 2.4 GHz peak clock?
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
cd /tmp && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5h
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc GRBM_COUNT GRBM_GUI_ACTIVE SQ_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $O/clk -o clk -- $GRAFT_REPO_ROOT/tools/gemm_exp/bin/gemm_exp_base 3 > $O/clk_run.log 2>&1 || { tail -20 $O/clk_run.log; exit 1; }
find $O/clk -name "*.csv" | head
