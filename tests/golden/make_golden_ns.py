"""Whole-solve golden fixtures at the north-star size, made by running the REFERENCE solvers.

Run in the build container only (the reference tree does not exist on the GPU box):

    OPENBLAS_NUM_THREADS=4 python tests/golden/make_golden_ns.py gl_ProxGD_primal
    OPENBLAS_NUM_THREADS=4 python tests/golden/make_golden_ns.py gl_FProxGD_primal

Each call solves (m, n, l) = (8192, 16384, 32), fp64, ``gen_data`` seed 97006855, with
``opts = {"alpha0": 1/(sqrt(m)+sqrt(n))^2}`` and every other option at the reference's
default (``code/gl_ProxGD_primal.py:10-19``, ``code/gl_FProxGD_primal.py:10-19``) through
the reference's own ``gl_<method>`` imported from ``/root/reference/code``.  That is
35-55 minutes of CPU per solver here (ProxGD 2176 s, FProxGD 3319 s at 4 BLAS threads).
It stores data only, in ``ns_<method>.npz`` / ``.json``:

- ``k``, ``fval``, ``f_hist``, ``f_hist_best`` of the reference run;
- the final iterate ``x``, as float32 (the test's bar on x is 1e-6 of max|x|; the fp64
  iterate's sha256 is in the .json);
- ``ns_instance_b.npz``: ``gen_data``'s ``b = A @ u`` goes through the host BLAS, whose
  summation order can differ between this container's CPU and the GPU box's, so the
  instance's right-hand side travels with the fixtures (A, u and x0 come from the portable
  MT19937 stream and are re-drawn by the test; their sha256 digests are stored to prove it).

``tests/test_gpu_ns_golden.py`` checks the HIP solvers against these files (VERDICT round 3,
"what's missing" item 2).
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

M, N, L, SEED = 8192, 16384, 32, 97006855


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main(method: str):
    import importlib
    import warnings
    warnings.simplefilter("ignore")
    solver = getattr(importlib.import_module(method), method)
    A, b, u, x0, mu = gen_data(M, N, L, SEED)
    opts = {"alpha0": step_size_for(M, N)}
    t0 = time.perf_counter()
    x, k, out = solver(x0, A, b, mu, dict(opts))
    secs = time.perf_counter() - t0
    f_hist = np.asarray([float(v) for v in out["f_hist"]], dtype=np.float64)
    f_best = np.asarray([float(v) for v in out["f_hist_best"]], dtype=np.float64)
    name = "ns_" + method
    x = np.asarray(x)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), x=x.astype(np.float32), f_hist=f_hist,
                        f_hist_best=f_best, k=np.int64(k), fval=np.float64(out["fval"]))
    np.savez_compressed(os.path.join(HERE, "ns_instance_b.npz"), b=b)   # same for both solvers
    meta = dict(solver=method, m=M, n=N, l=L, seed=SEED, dtype="f64", mu=mu, opts=opts,
                k=int(k), fval=float(out["fval"]), cpu_seconds=round(secs, 1),
                blas_threads=os.environ.get("OPENBLAS_NUM_THREADS"),
                sha256=dict(A=sha(A), x0=sha(x0), u=sha(u), b=sha(b)),
                x_sha256_f64=sha(x),
                x_stored_as="float32 (the test's bar on x is 1e-6 of max|x|)")
    with open(os.path.join(HERE, name + ".json"), "w") as fh:
        json.dump(meta, fh, indent=1, sort_keys=True)
    print("%-24s k=%5d fval=%.15e  %.0f s" % (name, k, float(out["fval"]), secs))


if __name__ == "__main__":
    main(sys.argv[1])
