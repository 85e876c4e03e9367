# round 6 call F: full GPU tier, smoke, --old-logp recompute bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/t_all.log 2>&1
rc=$?; tail -4 gpurun_out/t_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
tail -2 gpurun_out/smoke.log
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --skip-latency --old-logp recompute > gpurun_out/b_recompute.log 2>&1 || exit 1
grep "step " gpurun_out/b_recompute.log; tail -1 gpurun_out/b_recompute.log | grep -o '"value": [0-9.]*\|"behaviour_logp_gap": [0-9.e-]*\|"clipfrac_first_mb": [0-9.e-]*\|"phase_s_per_step": {[^}]*}\|"kl_ref_at_init": [0-9.e-]*'
