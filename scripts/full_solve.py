"""Whole-solve timing on the bench instance (same data as bench.py): runs the solver to its own
stop rule (or --maxit per phase) and prints one JSON line with k, tt, fval and iterations/s.
Used for A/B of solver modes over a complete trajectory (GLX_* knobs from the environment).

    python scripts/full_solve.py [--method gl_ProxGD_primal] [--m 8192 --n 16384 --l 32] [--maxit 0]
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

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--method", default="gl_ProxGD_primal")
    ap.add_argument("--m", type=int, default=8192)
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--l", type=int, default=32)
    ap.add_argument("--maxit", type=int, default=0, help="per phase (0 = the method's default)")
    ap.add_argument("--dtype", default="f64", choices=["f64", "f32"])
    a = ap.parse_args()
    import glx
    dev = torch.device("cuda", 0)
    dt = torch.float64 if a.dtype == "f64" else torch.float32
    A, b, x0 = bench.make_instance(a.m, a.n, a.l, 0, a.m, dt, dev)
    alpha0 = float(1.0 / (math.sqrt(a.m) + math.sqrt(a.n)) ** 2)
    opts = {"alpha0": alpha0}
    if a.maxit:
        opts["maxit"] = a.maxit
    # warm the clocks (bench.py's pre-warm), then the measured solve from x0
    glx.solve(a.method, x0.clone(), A, b, 1e-2, dict(opts, max_total_iters=500))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    x, k, out = glx.solve(a.method, x0.clone(), A, b, 1e-2, dict(opts))
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    print(json.dumps({"method": a.method, "dtype": a.dtype, "shape": [a.m, a.n, a.l], "k": int(k), "tt": out["tt"], "wall": wall,
                      "its": k / out["tt"], "fval": float(out["fval"]), "stats": out.get("stats"),
                      "ax_calls": out.get("ax_calls"), "ax_sources": out.get("ax_sources"),
                      "syncs": out.get("glx", {}).get("syncs"),
                      "env": {k2: v for k2, v in os.environ.items() if k2.startswith("GLX_")}}))


if __name__ == "__main__":
    main()
