"""Check that rocprofv3's kernel trace agrees with bench.py's live HIP-event timing.

    python scripts/prof_agree.py --trace DIR --bench bench.json [--out summary.json]

bench.py times the dense A@X, A^T R and (split-candidate) A e gather launches of the timed region
with HIP events on the solver's stream (every `timed_every`-th launch of each); the trace holds
every launch of the run. bench.py brackets its timed region with two marker kernels (torch's
spin kernel) launched outside it, so the trace's launches between the markers are exactly the
timed region's; their mean duration must agree with the events' (roofline.avg_launch_us,
atr_avg_launch_us, gather_avg_launch_us).
"""
import argparse
import csv
import glob
import json
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", required=True)
    ap.add_argument("--bench", required=True)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    bench = json.load(open(a.bench))
    roof = bench["roofline"]
    files = glob.glob(os.path.join(a.trace, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for f in files:
        rows += list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if "spin" in r["Kernel_Name"].lower() or "sleep" in r["Kernel_Name"].lower()]
    if len(marks) >= 2:
        region = rows[marks[-2] + 1:marks[-1]]
        how = "launches between the two marker kernels"
    else:
        region = None
        how = "no markers: the last launches_timed * timed_every launches of each kernel"
    out = {"bench_value": bench["value"], "bench_unit": bench["unit"], "region": how}
    for kind, key, tag in (("ax", "avg_launch_us", "k_ax_"), ("atr", "atr_avg_launch_us", "k_atr_"),
                           ("gather", "gather_avg_launch_us", "k_at_gather")):
        if roof.get(key) is None:
            continue
        src = region if region is not None else rows
        durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in src if tag in r["Kernel_Name"]]
        if region is None:
            n = roof.get("launches_timed", 0) * roof.get("timed_every", 1)
            durs = durs[-n:] if len(durs) >= n else durs
        avg = sum(durs) / max(1, len(durs))
        out[kind] = {"trace_launches": len(durs), "rocprof_avg_us": avg,
                     "bench_events_avg_us": roof[key], "ratio": avg / roof[key] if roof[key] else None}
    print(json.dumps(out, indent=1))
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
