"""Time the l = 16 one-pass trial batch + gradient (k_resgrad2) against the two-pass path
(A @ [X0 | X1], finalize, A^T R1) through glx_residual_gradient2, C2 shape by default. Run under
`rocprofv3 --kernel-trace --stats` for per-kernel durations (the one-pass call reads its error
flag back, so host-side timing includes a synchronisation)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "convex-optimization_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=4096)
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    from glx import kernels
    m, n = a.m, a.n
    A = torch.randn(m, n, device="cuda", dtype=torch.float64)
    X0 = torch.randn(n, 16, device="cuda", dtype=torch.float64)
    X1 = torch.randn(n, 16, device="cuda", dtype=torch.float64)
    B = torch.randn(m, 16, device="cuda", dtype=torch.float64)
    for one in (True, False):
        ran = None
        for _ in range(3):
            ran = kernels.residual_gradient2(A, X0, X1, B, one_pass=one)[3]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            kernels.residual_gradient2(A, X0, X1, B, one_pass=one)
        torch.cuda.synchronize()
        us = (time.perf_counter() - t0) / a.reps * 1e6
        print(json.dumps({"one_pass": one, "ran": ran, "host_us_per_call": round(us, 1)}), flush=True)


if __name__ == "__main__":
    main()
