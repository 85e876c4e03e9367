"""Per-phase kernel breakdown from a rocprofv3 run with --kernel-trace --marker-trace -f csv.

Usage: python tools/phase_breakdown.py <rocprof output dir> [--out summary.json] [--top 15]
Kernels are attributed to the innermost roctx range (PhaseTimer phases: rollout,
ref_logprobs+reward, update) whose time span contains the kernel's start timestamp.
"""
import argparse
import collections
import csv
import glob
import json
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("d")
    ap.add_argument("--out", default=None)
    ap.add_argument("--top", type=int, default=15)
    ap.add_argument("--grids", default="", help="comma-separated kernel-name substrings: per-phase grid-size "
                    "histogram (count, total ms) of those kernels, to tell which GEMM shapes ran where")
    a = ap.parse_args()
    kf = glob.glob(os.path.join(a.d, "**", "*kernel_trace.csv"), recursive=True)
    mf = glob.glob(os.path.join(a.d, "**", "*marker_api_trace.csv"), recursive=True)
    assert kf and mf, (kf, mf)
    ranges = []
    for r in csv.DictReader(open(mf[0])):
        try:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        except (KeyError, ValueError):
            continue
        name = r.get("Function") or r.get("Message") or r.get("Name") or ""
        if e > s:
            ranges.append((s, e, name))
    res = collections.defaultdict(lambda: collections.defaultdict(float))
    span = collections.defaultdict(float)
    want = [w for w in a.grids.split(",") if w]
    grids = collections.defaultdict(lambda: [0, 0.0])
    for r in csv.DictReader(open(kf[0])):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        best = None
        for (rs, re_, n) in ranges:
            if rs <= s <= re_ and (best is None or re_ - rs < best[1] - best[0]):
                best = (rs, re_, n)
        ph = best[2] if best else "(none)"
        res[ph][r["Kernel_Name"][:90]] += (e - s) / 1e6
        for w in want:
            if w in r["Kernel_Name"]:
                g = grids[(ph, w, r.get("Grid_Size_X", r.get("Grid_Size", "?")), r.get("Workgroup_Size_X", "?"))]
                g[0] += 1
                g[1] += (e - s) / 1e6
    count = collections.Counter()
    for (rs, re_, n) in ranges:
        span[n] += (re_ - rs) / 1e6
        count[n] += 1
    out = {}
    for ph, ks in res.items():
        tot = sum(ks.values())
        top = sorted(ks.items(), key=lambda x: -x[1])[: a.top]
        out[ph] = {"kernel_ms": tot, "wall_ms": span.get(ph, 0.0), "top": [[k, round(v, 3)] for k, v in top]}
        nr = max(count.get(ph, 1), 1)
        out[ph]["ranges"] = count.get(ph, 0)
        print(f"== {ph}: kernels {tot:.1f} ms / range {span.get(ph, 0.0):.1f} ms over {count.get(ph, 0)} range(s) "
              f"= {tot / nr:.1f} ms kernels per range")
        for k, v in top:
            print(f"   {v:8.2f} ms  {k}")
    for (ph, w, gx, wx), (n, ms) in sorted(grids.items(), key=lambda x: -x[1][1]):
        print(f"grid {ph:22s} {w:28s} grid_x={gx:>8} wg_x={wx:>4}  calls={n:6d}  {ms:9.2f} ms")
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
