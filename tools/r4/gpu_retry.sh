#!/bin/bash
# Retry a gpurun call only while the pool reports no free box / an infrastructure failure
# ("status=transient": the command never ran, nothing was charged). Any other outcome ends the loop.
#   tools/r4/gpu_retry.sh OUTFILE [ATTEMPTS] -- gpurun arguments...
out=$1; shift
n=30
if [ "$1" != "--" ] && [ "$1" -eq "$1" ] 2>/dev/null; then n=$1; shift; fi
[ "$1" = "--" ] && shift
for i in $(seq 1 "$n"); do
  /usr/local/graft/bin/gpurun "$@" > "$out" 2>&1
  if grep -q "status=transient" "$out"; then sleep 200; continue; fi
  break
done
