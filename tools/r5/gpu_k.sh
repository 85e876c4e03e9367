#!/bin/bash
# round 5, GPU call K: sampler timing probe (window path vs full-row search)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5k
mkdir -p $O
timeout -k 10 300 python -u tools/r5/sampler_probe.py > $O/sampler_probe.log 2>&1 || { tail -20 $O/sampler_probe.log; exit 1; }
cat $O/sampler_probe.log
