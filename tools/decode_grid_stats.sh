# Per-(kernel, grid) average durations of the batch-N decode loop (rocprofv3 kernel trace)
set -o pipefail
R=$PWD
N=${1:-1}
mkdir -p $R/gpurun_out/grid_dec$N
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/gd$N
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d /tmp/gd$N -o run -- python3 $R/tools/decode_profile.py --batch $N --prompt 173 --new 128 > $R/gpurun_out/grid_dec$N/log.txt 2>&1 || exit $?
f=$(find /tmp/gd$N -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'PY' > $R/gpurun_out/grid_dec$N/grid_stats.txt
import csv, sys, collections
acc = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    acc[(r["Kernel_Name"][:60], r.get("Grid_Size_X") or r.get("Grid_Size"), r.get("Workgroup_Size_X") or r.get("Workgroup_Size"))].append(
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
rows = sorted(acc.items(), key=lambda kv: -sum(kv[1]))
for (name, grid, wg), d in rows[:16]:
    d.sort()
    print(f"{name:60s} grid={grid:>8} wg={wg:>5} n={len(d):6d} med={d[len(d)//2]:8.2f}us total={sum(d)/1e3:8.1f}ms")
PY
rm -rf /tmp/gd$N
cat $R/gpurun_out/grid_dec$N/grid_stats.txt
