"""Time the fused residual-gradient pass (one read of A) against the two-pass path (A@X, then
A^T r) through the single-kernel C ABI, NS shape by default. Prints one JSON line per path."""
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
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=8192)
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    from glx import kernels
    m, n, l = a.m, a.n, 32
    A = torch.randn(m, n, device="cuda", dtype=torch.float64)
    X = torch.randn(n, l, device="cuda", dtype=torch.float64)
    B = torch.randn(m, l, device="cuda", dtype=torch.float64)
    flops = 4.0 * m * n * l
    us = timeit(lambda: kernels.residual_gradient(A, X, B, one_pass=True), a.reps)
    _, _, fused = kernels.residual_gradient(A, X, B, one_pass=True)
    print(json.dumps({"path": "fused" if fused else "two-pass(fallback)", "us": us,
                      "TFs": flops / us / 1e6, "frac_fp64": flops / us / 1e6 / 78.6}))
    def two():
        R, _ = kernels.residual(A, X, B)
        kernels.gradient(A, R)
    us2 = timeit(two, a.reps)
    print(json.dumps({"path": "two-pass", "us": us2, "TFs": flops / us2 / 1e6,
                      "frac_fp64": flops / us2 / 1e6 / 78.6}))


if __name__ == "__main__":
    main()
