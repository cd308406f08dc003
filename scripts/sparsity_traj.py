"""Sparsity trajectory of a whole solve on the bench instance: the fraction of nonzero entries of
the iterate after each iteration (the reference's sparsity_func, gl_ProxGD_primal.py:22), sampled.
Tells how much of A a support-restricted A@x would read over a solve.

    python scripts/sparsity_traj.py [--method gl_ProxGD_primal] [--m 8192 --n 16384 --l 32]
"""
import argparse
import json
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "convex-optimization_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--method", default="gl_ProxGD_primal")
    ap.add_argument("--m", type=int, default=8192)
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--l", type=int, default=32)
    a = ap.parse_args()
    import glx
    dev = torch.device("cuda", 0)
    A, b, x0 = bench.make_instance(a.m, a.n, a.l, 0, a.m, torch.float64, dev)
    alpha0 = float(1.0 / (math.sqrt(a.m) + math.sqrt(a.n)) ** 2)
    x = x0.clone()
    s = glx.Session(a.method, x, A, b, 1e-2, {"alpha0": alpha0})
    s.run(0)
    res = s.finish()
    sp, starts, breaks = s.trace()
    s.close()
    xr = x.abs().amax(dim=1)
    rows = int((xr > 1e-6 * float(xr.max())).sum())
    k = len(sp)
    idx = sorted(set([0, 5, 10, 25, 50, 100, 200, 400, 800, 1200, 1600, 2000, 2400, 2800, 3200,
                      4000, 5000, k - 1]))
    print(json.dumps({"method": a.method, "k": int(res["k"]), "phase_starts": list(starts),
                      "sparsity_after": {str(i): float(sp[i]) for i in idx if i < k},
                      "final_nonzero_rows": rows, "n": a.n}))


if __name__ == "__main__":
    main()
