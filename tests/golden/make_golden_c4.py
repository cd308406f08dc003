"""Whole-solve golden fixture for BASELINE config C4, made by running the REFERENCE solver.

Run in the build container only (the reference tree does not exist on the GPU box):

    OPENBLAS_NUM_THREADS=6 python tests/golden/make_golden_c4.py

``gl_SGD_primal`` fp64 at (m, n, l) = (65536, 8192, 1), ``gen_data`` seed 97006855, with
``opts = {"alpha0": 1/(sqrt(m)+sqrt(n))^2}`` and every other option at the reference's default,
through the reference's own ``gl_SGD_primal`` imported from ``/root/reference/code``. Stores
data only, in ``c4_gl_SGD_primal.npz`` / ``.json``: k, fval, f_hist, f_hist_best, the final
iterate (float32) and the instance's b (the host BLAS's ``A @ u`` is not portable bit for bit;
A, u and x0 are re-drawn by the test from the MT19937 stream, their sha256 stored).
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import time

import numpy as np

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/code"
sys.path.insert(0, ROOT)
sys.path.insert(0, REF)

from oracle.numpy_ref import gen_data, step_size_for  # noqa: E402

M, N, L, SEED = 65536, 8192, 1, 97006855


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main():
    import importlib
    import warnings
    warnings.simplefilter("ignore")
    method = "gl_SGD_primal"
    solver = getattr(importlib.import_module(method), method)
    A, b, u, x0, mu = gen_data(M, N, L, SEED)
    opts = {"alpha0": step_size_for(M, N)}
    t0 = time.perf_counter()
    x, k, out = solver(x0, A, b, mu, dict(opts))
    secs = time.perf_counter() - t0
    f_hist = np.asarray([float(v) for v in out["f_hist"]], dtype=np.float64)
    f_best = np.asarray([float(v) for v in out["f_hist_best"]], dtype=np.float64)
    name = "c4_" + method
    np.savez_compressed(os.path.join(HERE, name + ".npz"), x=np.asarray(x).astype(np.float32),
                        f_hist=f_hist, f_hist_best=f_best, k=np.int64(k), fval=np.float64(out["fval"]),
                        b=b)
    meta = dict(solver=method, m=M, n=N, l=L, seed=SEED, dtype="f64", mu=mu, opts=opts,
                k=int(k), fval=float(out["fval"]), cpu_seconds=round(secs, 1),
                blas_threads=os.environ.get("OPENBLAS_NUM_THREADS"),
                sha256=dict(A=sha(A), x0=sha(x0), u=sha(u), b=sha(b)))
    with open(os.path.join(HERE, name + ".json"), "w") as fh:
        json.dump(meta, fh, indent=1, sort_keys=True)
    print("%-24s k=%5d fval=%.15e  %.0f s" % (name, k, float(out["fval"]), secs))


if __name__ == "__main__":
    main()
