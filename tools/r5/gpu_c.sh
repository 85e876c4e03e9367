#!/bin/bash
# round 5, GPU call C: where the behaviour / target log-prob gap comes from at Mistral-7B shape
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5c
mkdir -p $O
timeout -k 10 600 python -u tools/r5/behaviour_gap_7b.py > $O/gap7b.log 2>&1 || { tail -30 $O/gap7b.log; exit 1; }
grep -v amdgpu.ids $O/gap7b.log
