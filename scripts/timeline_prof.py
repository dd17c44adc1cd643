"""GPU busy vs idle over the tail of a rocprofv3 kernel trace (the timed steps of a short bench run).

usage: python scripts/timeline_prof.py <kernel_trace.csv> [--last-ms 2400] [--gap-us 30]

Prints: the window's wall time, the union of kernel intervals (GPU busy), the idle time split by gap
size, the kernel pairs around the largest gaps, and busy time by kernel family (summarize_prof).
"""
import argparse
import collections
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from summarize_prof import FAMILIES  # noqa: E402


def family(name):
    for fam, f in FAMILIES:
        if f(name):
            return fam.split(" ")[0]
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last-ms", type=float, default=2400.0)
    ap.add_argument("--gap-us", type=float, default=30.0)
    ap.add_argument("--top", type=int, default=10)
    ap.add_argument("--marker", default=None,
                    help="kernel-name substring of a marker launched at the start and the end of the window "
                         "(bench.py GRAG_TRACE_MARK=1: a float64 fill); overrides --last-ms")
    a = ap.parse_args()
    ev = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    ev.sort()
    marks = [e for e in ev if a.marker and a.marker in e[2]]
    if len(marks) >= 2:
        t0, t_end = marks[0][1], marks[-1][0]
        ev = [e for e in ev if e[0] >= t0 and e[1] <= t_end and a.marker not in e[2]]
    else:
        t_end = max(e[1] for e in ev)
        t0 = t_end - int(a.last_ms * 1e6)
        ev = [e for e in ev if e[0] >= t0]
    busy = 0
    cur_s, cur_e = ev[0][0], ev[0][1]
    gaps = []
    prev_name = ev[0][2]
    fam_busy = collections.Counter()
    for s, e, n in ev:
        fam_busy[family(n)] += e - s
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, prev_name, n))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
        prev_name = n if e >= cur_e else prev_name
    busy += cur_e - cur_s
    wall = (t_end - t0) if len(marks) >= 2 else (t_end - ev[0][0])
    print(f"window {wall / 1e6:.1f} ms, kernels {len(ev)}, GPU busy {busy / 1e6:.1f} ms "
          f"({100 * busy / wall:.1f} %), idle {(wall - busy) / 1e6:.1f} ms")
    for lo, hi in ((0, 5), (5, 30), (30, 200), (200, 2000), (2000, 1e12)):
        g = [x for x in gaps if lo * 1e3 <= x[0] < hi * 1e3]
        print(f"  gaps {lo:>5}-{hi if hi < 1e12 else 'inf':>5} us: n={len(g):6d} total {sum(x[0] for x in g) / 1e6:8.2f} ms")
    pair = collections.Counter()
    pair_n = collections.Counter()
    for d, p, n in gaps:
        if d >= a.gap_us * 1e3:
            k = (p.split("(")[0][-60:], n.split("(")[0][-60:])
            pair[k] += d
            pair_n[k] += 1
    print(f"largest gap sources (gaps >= {a.gap_us} us, by total):")
    for k, v in pair.most_common(12):
        print(f"  {v / 1e6:8.2f} ms  n={pair_n[k]:5d}  {k[0]}  ->  {k[1]}")
    # the largest gaps with the kernels around them (times relative to the window start)
    idx = {id(e): i for i, e in enumerate(ev)}
    big = sorted(gaps, key=lambda g: -g[0])[: a.top]
    ends = []
    run_end = ev[0][1]
    for i, (s_, e_, n_) in enumerate(ev):
        if i and s_ > run_end:
            ends.append((s_ - run_end, i))
        run_end = max(run_end, e_)
    ends.sort(reverse=True)
    print(f"top {a.top} gaps with context:")
    for d, i in ends[: a.top]:
        print(f"  gap {d / 1e6:.2f} ms at t={(ev[i][0] - ev[0][0]) / 1e6:.1f} ms")
        for j in range(max(0, i - 4), min(len(ev), i + 3)):
            mark = ">>" if j == i else "  "
            print(f"    {mark} {(ev[j][0] - ev[0][0]) / 1e6:9.3f} +{(ev[j][1] - ev[j][0]) / 1e3:8.1f}us  "
                  f"{ev[j][2].split('(')[0][:90]}")
    del idx, big
    print("kernel time by family in the window:")
    for k, v in fam_busy.most_common():
        print(f"  {k:14s} {v / 1e6:8.1f} ms")


if __name__ == "__main__":
    main()
