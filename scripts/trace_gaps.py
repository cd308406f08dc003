"""Per-iteration kernel composition and inter-kernel gaps from a rocprofv3 kernel trace.

    python scripts/trace_gaps.py <kernel_trace.csv> [--last N]

Uses the last N kernel dispatches (the timed region of a bench run): busy time per kernel name,
the span, and the idle gaps between consecutive kernels (end of one to start of the next),
attributed to the kernel that follows the gap (median, so one-off setup gaps do not skew it).
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last", type=int, default=2000)
    ap.add_argument("--markers", action="store_true",
                    help="use the launches between the last two marker kernels (bench.py's timed region)")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
    marks = [i for i, k in enumerate(ks) if "spin" in k[2].lower() or "sleep" in k[2].lower()]
    if a.markers and len(marks) >= 2:
        ks = ks[marks[-2] + 1:marks[-1]]
    else:
        ks = ks[-a.last:]
    span = ks[-1][1] - ks[0][0]
    busy = collections.defaultdict(lambda: [0, 0])
    gaps = collections.defaultdict(list)
    for i, (s, e, n) in enumerate(ks):
        short = n.split("(")[0].split("<")[0][:40]
        busy[short][0] += 1
        busy[short][1] += e - s
        if i:
            g = s - ks[i - 1][1]
            gaps[short].append(max(g, 0))
    tot_busy = sum(v[1] for v in busy.values())
    print("kernels %d  span %.1f us  busy %.1f us (%.1f%%)" % (len(ks), span / 1e3, tot_busy / 1e3, 100 * tot_busy / span))
    for name, (c, t) in sorted(busy.items(), key=lambda kv: -kv[1][1]):
        g = sorted(gaps.get(name, [0]))
        print("%-42s calls %6d  avg %8.2f us  total %6.1f%%  gap-before median %6.2f us" %
              (name, c, t / c / 1e3, 100 * t / span, g[len(g) // 2] / 1e3))


if __name__ == "__main__":
    main()
