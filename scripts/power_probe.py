"""Probe: is the slow start of the NS bench (A@X 290 -> 417 -> 270 us over the first ~40
iterations) a power-management transient or data dependence (dense early iterates)?

    python scripts/power_probe.py [--reps 120]

Prints one JSON line per experiment with the per-launch times (us) of A @ [X1 | X2] (+ the
small finalize) for dense Gaussian X, all-zero X and 90 %-zero-row X, back to back, and then
the solver's own A@X launch times per iteration of a fresh Session from x0 (dense), run after
the GPU has been busy, and again after 2 s idle.
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "convex-optimization_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import make_instance  # noqa: E402


def series(fn, reps):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
    ev[0].record()
    for i in range(reps):
        fn()
        ev[i + 1].record()
    torch.cuda.synchronize()
    return [round(ev[i].elapsed_time(ev[i + 1]) * 1e3, 1) for i in range(reps)]


def session_series(A, b, x0, iters, label):
    import glx
    m, n = A.shape
    x = x0.clone()
    alpha0 = float(1.0 / (math.sqrt(m) + math.sqrt(n)) ** 2)
    s = glx.Session("gl_ProxGD_primal", x, A, b, 1e-2, {"alpha0": alpha0, "maxit": 2500,
                                                       "max_total_iters": iters + 2, "profile": 1})
    out = []
    for _ in range(iters):
        s.run(1)
        c, ms = s.kernel_time(0)
        out.append(round(ms / max(1, c) * 1e3, 1))
    s.close()
    print(json.dumps({"exp": label, "ax_us": out}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=120)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    from glx import kernels
    m, n, l = 8192, 16384, 32
    A, b, x0 = make_instance(m, n, l, 0, m, torch.float64, dev)
    torch.cuda.synchronize()
    time.sleep(2.0)
    session_series(A, b, x0, 60, "session_cold")
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    dense = [torch.randn(n, l, generator=g, device=dev, dtype=torch.float64) for _ in range(2)]
    zero = [torch.zeros(n, l, device=dev, dtype=torch.float64) for _ in range(2)]
    rowsp = [d.clone() for d in dense]
    keep = torch.rand(n, generator=g, device=dev) < 0.1
    for r in rowsp:
        r[~keep] = 0
    time.sleep(2.0)
    for label, X in (("dense", dense), ("zero", zero), ("rows10pct", rowsp), ("dense_again", dense)):
        t = series(lambda: kernels.residual_batch(A, X, b), a.reps)
        print(json.dumps({"exp": label, "us": t}), flush=True)
    session_series(A, b, x0, 60, "session_after_busy")
    time.sleep(2.0)
    session_series(A, b, x0, 60, "session_after_idle2s")


if __name__ == "__main__":
    main()
