#!/bin/bash
# round 5, GPU call T: config-5 decode path A/B (deferred W8A8 split-K vs reduced) on a 13B rollout
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5t
mkdir -p $O
timeout -k 10 900 python -u tools/r5/fp8_defer_probe.py > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
grep defer $O/probe.log
