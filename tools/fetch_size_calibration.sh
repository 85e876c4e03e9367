#!/bin/bash
# Calibrate rocprofv3 FETCH_SIZE against a known byte count (MI355X_MICROARCH.md: on gfx950 it reads
# half of a wide streaming read). tools/microbench/hbm_pattern.hip streams exactly 1 GiB per
# dispatch in three access patterns (16 rows x 128 B / 2 rows x 512 B / 1 row x 1 KiB per wave
# step); this records FETCH_SIZE per dispatch and prints bytes / (FETCH_SIZE x 1024).
# Usage (GPU box, repo root): bash tools/fetch_size_calibration.sh
set -o pipefail
R=$PWD
out=$R/gpurun_out/fetch_cal
mkdir -p $out
hipcc --offload-arch=gfx950 -O3 -o /tmp/hbm_pattern $R/tools/microbench/hbm_pattern.hip || exit 1
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/fsc
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d /tmp/fsc -o run -- /tmp/hbm_pattern > $out/run.log 2>&1 || exit $?
find /tmp/fsc -name "*counter_collection.csv" -exec cp {} $out/fetch.csv \;
rm -rf /tmp/fsc
python3 - "$out/fetch.csv" > $out/summary.txt <<'PY'
import collections, csv, statistics, sys
byts = 131072 * 4096 * 2  # one dispatch of hbm_pattern reads exactly this many bytes
v = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if r["Counter_Name"] == "FETCH_SIZE":
        v[(r["Kernel_Name"][:40], r.get("Grid_Size", "?"))].append(float(r["Counter_Value"]))
print(f"known bytes per dispatch: {byts}")
for k, xs in v.items():
    m = statistics.median(xs)
    print(f"{k[0]:40s} grid={k[1]:>8s} n={len(xs)} FETCH_SIZE={m:.0f} KB -> bytes/(FETCH_SIZE*1024) = {byts / (m * 1024):.3f}")
PY
cat $out/summary.txt
