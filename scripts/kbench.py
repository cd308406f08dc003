"""Sweep the A@x / A^T r kernel variants and split factors on the GPU (tuning tool).

    python scripts/kbench.py [--m 8192 --n 16384 --l 32] [--dtype f64] [--reps 20]

Prints one JSON line per (kernel, variant, split) with the average time per launch (HIP events
around `reps` back-to-back launches of the single-kernel C ABI, which adds the small residual
finalize kernel to A@x) and the algorithmic HBM rate s*(m*n + (m+n)*l) / t.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "convex-optimization_amd"))

import torch  # noqa: E402


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=8192)
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--l", type=int, default=32)
    ap.add_argument("--dtype", default="f64")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--ax", default="141,142,143,121,122,123,241,242")
    ap.add_argument("--atr", default="101,102,103,104,111,112,114")
    ap.add_argument("--splits", default="0,1,2,4,8,16")
    ap.add_argument("--axb", default="", help="batched (2-RHS) variants, e.g. 2420,1420,2220")
    ap.add_argument("--axb3", default="", help="batched (3-RHS) variants")
    ap.add_argument("--no-ref", action="store_true", help="skip the torch streaming reference")
    args = ap.parse_args()
    from glx import kernels
    dt = torch.float64 if args.dtype == "f64" else torch.float32
    es = 8 if args.dtype == "f64" else 4
    m, n, l = args.m, args.n, args.l
    A = torch.randn(m, n, device="cuda", dtype=dt)
    X = torch.randn(n, l, device="cuda", dtype=dt)
    B = torch.randn(m, l, device="cuda", dtype=dt)
    R = torch.randn(m, l, device="cuda", dtype=dt)
    nbytes = es * (m * n + (m + n) * l)
    ref_r = (A.double() @ X.double() - B.double())
    ref_g = A.double().T @ R.double()
    for v in [int(s) for s in args.ax.split(",") if s]:
        for S in [int(s) for s in args.splits.split(",")]:
            os.environ["GLX_AX_S"] = str(S)
            got, _ = kernels.residual(A, X, B, variant=v)
            err = float((got.double() - ref_r).abs().max() / ref_r.abs().max())
            t = timeit(lambda: kernels.residual(A, X, B, variant=v), args.reps)
            print(json.dumps({"kernel": "ax", "variant": v, "split": S, "us": t * 1e6,
                              "GBs": nbytes / t / 1e9, "relerr": err, "dtype": args.dtype,
                              "shape": [m, n, l]}), flush=True)
    for nsrc, codes in ((2, args.axb), (3, args.axb3)):
        if not codes:
            continue
        Xs = [X] + [torch.randn(n, l, device="cuda", dtype=dt) for _ in range(nsrc - 1)]
        refs = [(A.double() @ x.double() - B.double()) for x in Xs]
        nb = es * (m * n + (m + n) * l * nsrc)
        for v in [int(s) for s in codes.split(",") if s]:
            for S in [int(s) for s in args.splits.split(",")]:
                os.environ["GLX_AXB_VARIANT"] = str(v)
                os.environ["GLX_AX_S"] = str(S)
                os.environ["GLX_AXB_S"] = str(S)   # kind-5 (LDS) tiles take their own split
                Rs, _ = kernels.residual_batch(A, Xs, B)
                err = max(float((r.double() - rf).abs().max() / rf.abs().max()) for r, rf in zip(Rs, refs))
                t = timeit(lambda: kernels.residual_batch(A, Xs, B), args.reps)
                print(json.dumps({"kernel": "ax_batch%d" % nsrc, "variant": v, "split": S,
                                  "us": t * 1e6, "GBs": nb / t / 1e9,
                                  "TFs": 2.0 * m * n * l * nsrc / t / 1e12, "relerr": err,
                                  "dtype": args.dtype, "shape": [m, n, l]}), flush=True)
    os.environ["GLX_AX_S"] = "0"
    os.environ["GLX_AXB_S"] = "0"
    for v in [int(s) for s in args.atr.split(",") if s]:
        for S in [int(s) for s in args.splits.split(",")]:
            os.environ["GLX_ATR_VARIANT"] = str(v)
            os.environ["GLX_ATR_S"] = str(S)
            got = kernels.gradient(A, R)
            err = float((got.double() - ref_g).abs().max() / ref_g.abs().max())
            t = timeit(lambda: kernels.gradient(A, R), args.reps)
            print(json.dumps({"kernel": "atr", "variant": v, "split": S, "us": t * 1e6,
                              "GBs": nbytes / t / 1e9, "relerr": err, "dtype": args.dtype,
                              "shape": [m, n, l]}), flush=True)
    if args.no_ref:
        return
    # plain streaming reference: read A once with torch (sum) to calibrate achievable HBM
    t = timeit(lambda: A.sum(), args.reps)
    print(json.dumps({"kernel": "torch_sum_A", "us": t * 1e6, "GBs": es * m * n / t / 1e9}), flush=True)
    t = timeit(lambda: A.clone(), 5)
    print(json.dumps({"kernel": "torch_clone_A", "us": t * 1e6, "GBs": 2 * es * m * n / t / 1e9}), flush=True)


if __name__ == "__main__":
    main()
