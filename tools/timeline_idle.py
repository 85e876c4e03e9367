"""GPU idle time in a rocprofv3 trace: merges the busy intervals of every queue's kernels and copies,
then lists the idle gaps above a threshold with the work on either side and the roctx range they
fall in — where a step leaves the GPU waiting on the host.

    python tools/timeline_idle.py <dir with *kernel_trace.csv [*marker_api_trace.csv *memory_copy_trace.csv]>
        [--min-gap-ms 0.5] [--last-frac 0.5]
"""
import argparse
import csv
import glob
import os


def short(n):
    return n.split("(")[0].replace("void ", "").replace("rt::gb::", "").replace("rt::", "")[:50]


def load(d, pat):
    out = []
    for f in glob.glob(os.path.join(d, "**", pat), recursive=True):
        out += list(csv.DictReader(open(f)))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--min-gap-ms", type=float, default=0.5)
    ap.add_argument("--last-frac", type=float, default=0.5, help="analyse this trailing fraction of the run")
    a = ap.parse_args()
    ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]))
          for r in load(a.dir, "*kernel_trace.csv")]
    ev += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy:" + r.get("Direction", "?"))
           for r in load(a.dir, "*memory_copy_trace.csv")]
    ev.sort()
    t_first, t_last = ev[0][0], max(e for _, e, _ in ev)
    t_from = t_last - (t_last - t_first) * a.last_frac
    ev = [x for x in ev if x[0] >= t_from]
    ranges = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Function") or r.get("Message") or r.get("Name") or "")
              for r in load(a.dir, "*marker_api_trace.csv")]

    def where(t):
        hits = [n for s, e, n in ranges if s <= t <= e]
        return "/".join(hits[-2:]) if hits else "-"

    busy, gaps = 0, []
    cur_s, cur_e, last_name = ev[0][0], ev[0][1], ev[0][2]
    for s, e, n in ev[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, cur_e, last_name, n))
            cur_s, cur_e = s, e
        elif e > cur_e:
            cur_e = e
        if e >= cur_e:
            last_name = n
    busy += cur_e - cur_s
    span = ev[-1][1] - ev[0][0]
    idle = span - busy
    print(f"window {span / 1e6:.1f} ms  busy {busy / 1e6:.1f} ms  idle {idle / 1e6:.1f} ms ({100 * idle / span:.1f} %)")
    big = [g for g in gaps if g[0] >= a.min_gap_ms * 1e6]
    print(f"gaps >= {a.min_gap_ms} ms: {len(big)} totalling {sum(g[0] for g in big) / 1e6:.1f} ms; "
          f"smaller gaps total {(idle - sum(g[0] for g in big)) / 1e6:.1f} ms over {len(gaps) - len(big)}")
    for g, t, before, after in sorted(big, reverse=True)[:40]:
        print(f"{g / 1e6:8.2f} ms at +{(t - ev[0][0]) / 1e6:9.1f} ms  [{where(t)}]  {before} -> {after}")


if __name__ == "__main__":
    main()
