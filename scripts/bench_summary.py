"""One-line summary of bench.py JSON lines (round 5 scripts): it/s, per-kernel event averages,
flagged rows per trial, the whole solve and its check against the reference run."""
import json
import sys

for path in sys.argv[1:]:
    d = json.loads([x for x in open(path) if x.startswith("{")][-1])
    r = d["roofline"]
    k = r.get("kernels", {})
    w = d.get("whole_solve") or {}
    v = w.get("vs_reference") or {}
    print("%s %.1f it/s ax %.1f atr %.1f gather %.1f rows %.0f | whole k=%s %.1f it/s fval %s ref_ok=%s (f_hist %s)" % (
        path, d["value"], (k.get("ax") or {}).get("avg_launch_us") or 0,
        (k.get("atr") or {}).get("avg_launch_us") or 0, r.get("gather_avg_launch_us") or 0,
        r.get("sparse_rows_per_launch") or 0, w.get("k"), w.get("iters_per_s") or 0, w.get("fval"),
        v.get("within_bar"), v.get("f_hist_max_rel_diff")))
