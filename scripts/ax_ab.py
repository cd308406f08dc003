"""Interleaved A/B of A@X tiles (tuning tool, run under rocprofv3 --kernel-trace).

    rocprofv3 --kernel-trace --output-format csv -d OUT -o run -- \
        python scripts/ax_ab.py --codes 51328,83208 --env GLX_AX_ROT=0,1 --order OUT/order.json
    python scripts/ax_ab.py --summarize OUT

After a pre-warm (the MI355X clocks down over the first milliseconds of an fp64 MFMA load,
DESIGN.md (d)), every (tile code, env setting) runs `reps` launches per round, rounds
interleaved, so slow drifts hit every arm alike. --order writes the launch order; --summarize
matches it against the kernel trace (one A@X kernel per call) and prints each arm's median and
minimum kernel time and the algorithmic HBM rate s*(m*n + (m+n)*l*nsrc) / t.
"""
import argparse
import csv
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "convex-optimization_amd"))


def run(a):
    import torch
    from glx import kernels
    m, n, l = a.m, a.n, a.l
    dt = torch.float64 if a.dtype == "f64" else torch.float32
    A = torch.randn(m, n, device="cuda", dtype=dt)
    Xs = [torch.randn(n, l, device="cuda", dtype=dt) for _ in range(a.nsrc)]
    B = torch.randn(m, l, device="cuda", dtype=dt)
    codes = [int(c) for c in a.codes.split(",") if c]
    key, vals = (a.env.split("=") + [""])[:2] if a.env else ("", "")
    vals = vals.split(",") if key else [None]
    arms = [(c, v) for c in codes for v in vals]

    def call(code, v):
        if key:
            os.environ[key] = v
        if a.nsrc == 1:
            kernels.residual(A, Xs[0], B, variant=code)
        else:
            os.environ["GLX_AXB_VARIANT"] = str(code)
            kernels.residual_batch(A, Xs, B)

    order = []
    t0 = time.time()
    npw = 0
    while time.time() - t0 < a.prewarm:
        call(*arms[0])
        npw += 1
        if npw % 20 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    order.append(["prewarm", npw])
    for r in range(a.rounds):
        for c, v in arms:
            for _ in range(a.reps):
                call(c, v)
            torch.cuda.synchronize()
            order.append(["%d%s" % (c, ("/%s=%s" % (key, v)) if key else ""), a.reps])
    with open(a.order, "w") as fh:
        json.dump({"order": order, "shape": [m, n, l], "nsrc": a.nsrc, "dtype": a.dtype}, fh)


def summarize(d):
    meta = json.load(open(os.path.join(d, "order.json")))
    m, n, l = meta["shape"]
    es = 8 if meta["dtype"] == "f64" else 4
    nb = es * (m * n + (m + n) * l * meta["nsrc"])
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f)) if "k_ax_" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    i = 0
    arms = {}
    names = {}
    for label, cnt in meta["order"]:
        seg = rows[i:i + cnt]
        i += cnt
        if label == "prewarm":
            continue
        arms.setdefault(label, []).extend(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in seg)
        names[label] = seg[0]["Kernel_Name"].split("(")[0][:90] if seg else "?"
    out = []
    for label, v in arms.items():
        v = sorted(v)
        med = v[len(v) // 2]
        out.append({"arm": label, "kernel": names[label], "median_us": round(med, 2),
                    "min_us": round(v[0], 2), "n": len(v), "TBs_median": round(nb / med / 1e6, 3)})
    for o in sorted(out, key=lambda o: o["median_us"]):
        print(json.dumps(o))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=8192)
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--l", type=int, default=32)
    ap.add_argument("--dtype", default="f64")
    ap.add_argument("--nsrc", type=int, default=1)
    ap.add_argument("--codes", default="51328")
    ap.add_argument("--env", default="", help="NAME=v1,v2: A/B an environment knob")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--prewarm", type=float, default=1.5)
    ap.add_argument("--order", default="order.json")
    ap.add_argument("--summarize", default="")
    a = ap.parse_args()
    if a.summarize:
        summarize(a.summarize)
    else:
        run(a)
