# A/B of non-temporal weight (RT_GEMM_B_NT) and K/V (RT_ATTN_KV_NT) loads in the batch-256 decode
# loop: per-kernel statistics of each setting -> gpurun_out/nt_ab/<gemm>_<kv>_kernel_stats.csv
set -o pipefail
R=$PWD
mkdir -p $R/gpurun_out/nt_ab
cd /tmp && export TMPDIR=/tmp
for v in "0 0" "1 1" "0 0" "1 1"; do
  set -- $v
  rm -rf /tmp/ntab
  RT_GEMM_B_NT=$1 RT_ATTN_KV_NT=$2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d /tmp/ntab -o run -- \
    python3 $R/tools/decode_profile.py --batch 256 --prompt 173 --new 128 > $R/gpurun_out/nt_ab/log_$1_$2.txt 2>&1 || exit $?
  find /tmp/ntab -name "*kernel_stats.csv" -exec cp {} $R/gpurun_out/nt_ab/$1_$2_kernel_stats.csv \;
  python3 - "$R/gpurun_out/nt_ab/$1_$2_kernel_stats.csv" "$1" "$2" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:6]:
    print(f"gemm_nt={sys.argv[2]} kv_nt={sys.argv[3]} {r['Name'][:60]:60s} {float(r['AverageNs'])/1e3:8.2f} us x {r['Calls']}")
PY
done
