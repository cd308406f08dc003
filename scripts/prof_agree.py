"""Check that rocprofv3's kernel trace agrees with bench.py's live HIP-event timing.

    python scripts/prof_agree.py --trace DIR --bench bench.json [--out summary.json]

bench.py times the A@X and A^T R launches of the timed region with HIP events on the solver's
stream (every `timed_every`-th launch); the trace holds every launch of the run (warmup
included). The last launches_timed * timed_every A@X dispatches of the trace are the timed
region's; their mean duration must agree with roofline.avg_launch_us (and likewise A^T R).
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
    out = {"bench_value": bench["value"], "bench_unit": bench["unit"]}
    for kind, key, tag in (("ax", "avg_launch_us", "k_ax_"), ("atr", "atr_avg_launch_us", "k_atr_")):
        durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if tag in r["Kernel_Name"]]
        n = roof.get("launches_timed", roof.get("launches", 0)) * roof.get("timed_every", 1)
        tail = durs[-n:] if len(durs) >= n else durs
        avg = sum(tail) / max(1, len(tail))
        out[kind] = {"trace_launches": len(durs), "compared": len(tail), "rocprof_avg_us": avg,
                     "bench_events_avg_us": roof[key], "ratio": avg / roof[key] if roof[key] else None}
    print(json.dumps(out, indent=1))
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
