#!/bin/bash
# round 5, GPU call M: clock and instruction mix of the batch-1 sampler (PMC per dispatch)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
cd /tmp && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5m
mkdir -p $O
timeout -s KILL 60 rocprofv3 --pmc GRBM_COUNT GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $O/pmc -o p -- $GRAFT_REPO_ROOT/tools/sampler_exp/bin/sampler_exp_full 1 1.3 > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 1; }
python3 - <<'PY'
import csv, collections, statistics, os
d=os.environ['GRAFT_REPO_ROOT']+'/gpurun_out/r5m/pmc'
cc=list(csv.DictReader(open(d+'/p_counter_collection.csv')))
kt=list(csv.DictReader(open(d+'/p_kernel_trace.csv')))
dur={r['Dispatch_Id']:(int(r['End_Timestamp'])-int(r['Start_Timestamp']), r['Kernel_Name']) for r in kt}
vals=collections.defaultdict(dict)
for r in cc: vals[r['Dispatch_Id']][r['Counter_Name']]=float(r['Counter_Value'])
rows=[(dur[k][0], v) for k,v in vals.items() if k in dur and 'topk' in dur[k][1]]
print('dispatches', len(rows))
for key in sorted(rows[0][1]):
    print(key, statistics.median([v[key] for _,v in rows]))
print('dur_ns', statistics.median([a for a,_ in rows]))
PY
