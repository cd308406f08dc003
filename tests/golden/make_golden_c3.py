"""Whole-solve golden fixture for BASELINE config C3, made by running the REFERENCE solver.

Run in the build container only (the reference tree does not exist on the GPU box):

    OPENBLAS_NUM_THREADS=6 python tests/golden/make_golden_c3.py

``gl_FProxGD_primal`` in fp32 at (m, n, l) = (8192, 16384, 32): ``gen_data`` seed 97006855
(A, u, x0 re-drawn from the portable MT19937 stream, b from ``ns_instance_b.npz`` as in
``make_golden_ns.py``), all cast to float32, ``opts = {"alpha0": 1/(sqrt(m)+sqrt(n))^2}`` and
every other option at the reference's default, through the reference's own
``gl_FProxGD_primal`` imported from ``/root/reference/code``. It stores data only, in
``c3_gl_FProxGD_primal.npz`` / ``.json``: k, fval, f_hist, f_hist_best of the reference run and
its final iterate (float32). ``tests/test_gpu_ns_golden.py`` checks the HIP solver's fp32 path
(round 4: the split-candidate batch and the f32 LDS-DMA tile) against it.
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


def main():
    import importlib
    import warnings
    warnings.simplefilter("ignore")
    method = "gl_FProxGD_primal"
    solver = getattr(importlib.import_module(method), method)
    A, _, u, x0, mu = gen_data(M, N, L, SEED)
    b = np.load(os.path.join(HERE, "ns_instance_b.npz"))["b"]
    A32, b32, x032 = (a.astype(np.float32) for a in (A, b, x0))
    del A
    opts = {"alpha0": step_size_for(M, N)}
    t0 = time.perf_counter()
    x, k, out = solver(x032, A32, b32, mu, dict(opts))
    secs = time.perf_counter() - t0
    f_hist = np.asarray([float(v) for v in out["f_hist"]], dtype=np.float64)
    f_best = np.asarray([float(v) for v in out["f_hist_best"]], dtype=np.float64)
    name = "c3_" + method
    x = np.asarray(x, dtype=np.float32)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), x=x, f_hist=f_hist, f_hist_best=f_best,
                        k=np.int64(k), fval=np.float64(out["fval"]))
    meta = dict(solver=method, m=M, n=N, l=L, seed=SEED, dtype="f32", mu=mu, opts=opts,
                k=int(k), fval=float(out["fval"]), cpu_seconds=round(secs, 1),
                blas_threads=os.environ.get("OPENBLAS_NUM_THREADS"),
                sha256=dict(A32=sha(A32), x032=sha(x032), b32=sha(b32)))
    with open(os.path.join(HERE, name + ".json"), "w") as fh:
        json.dump(meta, fh, indent=1, sort_keys=True)
    print("%-24s k=%5d fval=%.15e  %.0f s" % (name, k, float(out["fval"]), secs))


if __name__ == "__main__":
    main()
