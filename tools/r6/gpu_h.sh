# round 6 call H: rocprofv3 kernel profiles of the final tree — one PPO step range-attributed to
# its phases (roctx markers), and the batch-1 RAG answer loop
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6prof
mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv -d /tmp/profppo -o run -- python3 -u bench.py --steps 2 --warmup 1 --skip-latency > $O/ppo_bench.log 2>&1 || { tail -20 $O/ppo_bench.log; exit 1; }
find /tmp/profppo -name "*kernel_stats.csv" -exec cp {} $O/ppo_kernel_stats.csv \;
python3 tools/phase_breakdown.py /tmp/profppo --out $O/ppo_phases.json --top 25 > $O/ppo_phases.txt 2>&1 || { tail -20 $O/ppo_phases.txt; exit 1; }
head -5 $O/ppo_phases.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/profb1 -o run -- python3 -u bench.py --steps 0 --latency-queries 16 > $O/b1_bench.log 2>&1 || { tail -20 $O/b1_bench.log; exit 1; }
find /tmp/profb1 -name "*kernel_stats.csv" -exec cp {} $O/b1_kernel_stats.csv \;
head -12 $O/b1_kernel_stats.csv | cut -c1-160
