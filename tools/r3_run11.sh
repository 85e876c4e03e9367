#!/bin/bash
# Wide W8A16 kernel split-K sweep (non-power-of-two splits) at decode M = 24..64.
set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 500 python3 -u tools/fp8_decode_table.py --ms 32,64 --splits 2,3,4,6,8,10,12,16 > gpurun_out/r3/fp8_split_sweep.log 2>&1 || { tail -20 gpurun_out/r3/fp8_split_sweep.log; exit 1; }
grep -v "^/opt" gpurun_out/r3/fp8_split_sweep.log | python3 -c "
import json,sys
for l in sys.stdin:
    if l.startswith('{\"kind'):
        r=json.loads(l); print(r['model'],r['name'],r['M'],'bf16',r['bf16_us'],'fp8',r['fp8_us'],r.get('fp8_split_us'))
"
