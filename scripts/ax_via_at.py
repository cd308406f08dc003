"""A @ X at the north-star shape two ways: the A@X tile over A (glx_residual, incl. its finalize)
and the A^T R panel kernel over the transposed copy At = A^T (glx_gradient(At, X) = At^T X =
A X), whose loads are contiguous 256-B pieces with the non-temporal policy. Prints per-call
times (HIP events, 20 calls after 3 warm) and the max relative difference of the two products.

    python scripts/ax_via_at.py            (GLX_ATR_S=<k> to force the panel kernel's row splits)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "convex-optimization_amd"))

import torch  # noqa: E402


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for e0, e1 in ev:
        e0.record()
        fn()
        e1.record()
    torch.cuda.synchronize()
    ts = sorted(e0.elapsed_time(e1) * 1e3 for e0, e1 in ev)
    return ts[0], ts[len(ts) // 2]


def main():
    from glx import kernels
    m, n, l = 8192, 16384, 32
    g = torch.Generator(device="cuda").manual_seed(0)
    A = torch.randn(m, n, dtype=torch.float64, device="cuda", generator=g)
    X = torch.randn(n, l, dtype=torch.float64, device="cuda", generator=g)
    B = torch.zeros(m, l, dtype=torch.float64, device="cuda")
    At = A.t().contiguous()
    R, _ = kernels.residual(A, X, B)
    P = kernels.gradient(At, X)
    rel = float((R - P).abs().max() / R.abs().max())
    b_ax = timed(lambda: kernels.residual(A, X, B))
    b_at = timed(lambda: kernels.gradient(At, X))
    gb = m * n * 8 / 1e9
    print(json.dumps({"ax_tile_us": b_ax, "at_panel_us": b_at, "rel_diff": rel,
                      "at_panel_TBps_best": gb / b_at[0] * 1e3,
                      "env": {k: v for k, v in os.environ.items() if k.startswith("GLX_")}}))


if __name__ == "__main__":
    main()
