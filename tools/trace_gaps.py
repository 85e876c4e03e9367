"""Idle time between consecutive kernels of a rocprofv3 kernel trace (one queue), summarised per
kernel pair over the steady-state window: how much of a decode step is launch / ramp bubbles.

    python tools/trace_gaps.py <kernel_trace.csv> [--top 15] [--skip-frac 0.3]
"""
import argparse
import csv
import collections


def short(n):
    n = n.split("(")[0]
    return n.replace("void ", "").replace("rt::gb::", "").replace("rt::", "")[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--top", type=int, default=15)
    ap.add_argument("--skip-frac", type=float, default=0.3, help="drop this leading fraction of dispatches")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[int(len(rows) * a.skip_frac):]
    busy = 0
    gaps = collections.defaultdict(list)
    durs = collections.defaultdict(list)
    prev = None
    total_gap = 0
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = short(r["Kernel_Name"])
        durs[name].append(e - s)
        busy += e - s
        if prev is not None:
            g = s - prev[1]
            if 0 <= g < 50_000:  # ignore host-side pauses between generations
                gaps[(prev[0], name)].append(g)
                total_gap += g
        prev = (name, e)
    print(f"dispatches {len(rows)}  kernel time {busy / 1e6:.2f} ms  inter-kernel gaps (<50 us) {total_gap / 1e6:.2f} ms")
    print("-- mean duration per kernel")
    for n, d in sorted(durs.items(), key=lambda kv: -sum(kv[1]))[: a.top]:
        print(f"  {sum(d) / 1e6:9.2f} ms  n={len(d):6d}  mean {sum(d) / len(d) / 1e3:8.2f} us  {n}")
    print("-- gaps per kernel pair")
    for k, g in sorted(gaps.items(), key=lambda kv: -sum(kv[1]))[: a.top]:
        print(f"  {sum(g) / 1e6:9.2f} ms  n={len(g):6d}  mean {sum(g) / len(g) / 1e3:6.2f} us  {k[0]} -> {k[1]}")


if __name__ == "__main__":
    main()
