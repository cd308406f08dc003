"""Generate the golden fixtures in tests/golden/ by running the REFERENCE solvers.

Run in the build container only (the reference tree does not exist on the GPU box):

    python tests/golden/make_golden.py

It imports ``gl_*_primal`` from ``/root/reference/code`` (read-only tree, so byte-code
writing is disabled), feeds them instances built by the repo's own generator
(``oracle.numpy_ref.gen_data`` — a restatement of ``main.py:37-51``) and stores only
data: input hashes, iteration counts, objective histories and final iterates.  No
reference source is copied.  ``tests/test_oracle.py`` checks the oracle against these
files; ``tests/test_gpu_parity.py`` checks the HIP path against them.
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/code"
sys.path.insert(0, ROOT)
sys.path.insert(0, REF)

from oracle.numpy_ref import gen_data, step_size_for  # noqa: E402

import gl_ProxGD_primal as _p  # noqa: E402
import gl_FProxGD_primal as _f  # noqa: E402
import gl_SGD_primal as _s  # noqa: E402
import gl_GD_primal as _g  # noqa: E402
import gl_FGD_primal as _fg  # noqa: E402

REF_SOLVERS = {
    "gl_ProxGD_primal": _p.gl_ProxGD_primal,
    "gl_FProxGD_primal": _f.gl_FProxGD_primal,
    "gl_SGD_primal": _s.gl_SGD_primal,
    "gl_GD_primal": _g.gl_GD_primal,
    "gl_FGD_primal": _fg.gl_FGD_primal,
}


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


# (case name, solver, (m, n, l), seed, dtype, opts)
CASES = []
DEF = (256, 512, 2)
for s in REF_SOLVERS:
    CASES.append(("default_" + s, s, DEF, 97006855, "f64", {}))
for s in ("gl_ProxGD_primal", "gl_FProxGD_primal"):
    for it in (1, 2, 5):
        CASES.append(("short%d_%s" % (it, s), s, DEF, 97006855, "f64", {"maxit": it}))
CASES.append(("seed114514_gl_SGD_primal", "gl_SGD_primal", DEF, 114514, "f64", {}))
CASES.append(("seed114514_gl_ProxGD_primal", "gl_ProxGD_primal", DEF, 114514, "f64", {}))
# BASELINE config C1 shape: default opts diverge for ProxGD (NaN), FProxGD survives
CASES.append(("c1_nan_gl_ProxGD_primal", "gl_ProxGD_primal", (512, 1024, 2), 97006855, "f64", {}))
CASES.append(("c1_gl_FProxGD_primal", "gl_FProxGD_primal", (512, 1024, 2), 97006855, "f64", {}))
CASES.append(("c1_conv_gl_ProxGD_primal", "gl_ProxGD_primal", (512, 1024, 2), 97006855, "f64",
              {"alpha0": 1.9 * step_size_for(512, 1024), "maxit": 10000}))
# mid-size, l=8 (VALU path) and the MFMA shapes (l = 16, 32), fp64 and fp32
for (shape, dt) in [((1024, 2048, 8), "f64"), ((1024, 2048, 8), "f32"),
                    ((512, 1024, 16), "f64"), ((256, 512, 32), "f64"), ((256, 512, 32), "f32"),
                    ((384, 640, 16), "f32")]:
    m, n, l = shape
    for s in ("gl_ProxGD_primal", "gl_FProxGD_primal"):
        CASES.append(("mid_%dx%dx%d_%s_%s" % (m, n, l, dt, s), s, shape, 1234 + l, dt,
                      {"alpha0": step_size_for(m, n), "maxit": 40}))
# tall GEMV (BASELINE config C4 shape family), SGD l=1
CASES.append(("tall_gl_SGD_primal", "gl_SGD_primal", (2048, 256, 1), 4242, "f64",
              {"alpha0": step_size_for(2048, 256), "maxit": 60}))
CASES.append(("tall_gl_GD_primal", "gl_GD_primal", (2048, 256, 1), 4242, "f64",
              {"alpha0": step_size_for(2048, 256), "maxit": 60}))
# ragged shapes (nothing a multiple of a tile)
CASES.append(("ragged_gl_ProxGD_primal", "gl_ProxGD_primal", (301, 517, 3), 77, "f64",
              {"alpha0": step_size_for(301, 517), "maxit": 50}))
CASES.append(("ragged_gl_FProxGD_primal", "gl_FProxGD_primal", (333, 250, 17), 78, "f64",
              {"alpha0": step_size_for(333, 250), "maxit": 50}))
CASES.append(("ragged_gl_SGD_primal", "gl_SGD_primal", (301, 517, 3), 79, "f64",
              {"alpha0": step_size_for(301, 517), "maxit": 30}))
for s in ("gl_FGD_primal", "gl_GD_primal", "gl_SGD_primal"):
    for it in (3, 40):
        CASES.append(("short%d_%s" % (it, s), s, DEF, 97006855, "f64", {"maxit": it}))
CASES.append(("mid_512x1024x16_f64_gl_FGD_primal", "gl_FGD_primal", (512, 1024, 16), 1250, "f64",
              {"alpha0": step_size_for(512, 1024), "maxit": 40}))
CASES.append(("mid_256x512x32_f32_gl_SGD_primal", "gl_SGD_primal", (256, 512, 32), 1266, "f32",
              {"alpha0": step_size_for(256, 512), "maxit": 40, "step_type": "fixed"}))
CASES.append(("steps_fixed_gl_ProxGD_primal", "gl_ProxGD_primal", DEF, 97006855, "f64",
              {"step_type": "fixed", "maxit": 100}))
CASES.append(("steps_dim_gl_FProxGD_primal", "gl_FProxGD_primal", DEF, 97006855, "f64",
              {"step_type": "diminishing", "maxit": 1100}))


def main():
    import warnings
    warnings.simplefilter("ignore")
    index = {}
    for name, solver, (m, n, l), seed, dt, opts in CASES:
        A, b, u, x0, mu = gen_data(m, n, l, seed)
        if dt == "f32":
            A, b, u, x0 = (a.astype(np.float32) for a in (A, b, u, x0))
        x, k, out = REF_SOLVERS[solver](x0, A, b, mu, dict(opts))
        f_hist = np.asarray([float(v) for v in out["f_hist"]], dtype=np.float64)
        f_best = np.asarray([float(v) for v in out["f_hist_best"]], dtype=np.float64)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), x=np.asarray(x), f_hist=f_hist,
                            f_hist_best=f_best, k=np.int64(k), fval=np.float64(out["fval"]))
        index[name] = dict(solver=solver, m=m, n=n, l=l, seed=seed, dtype=dt, mu=mu, opts=opts,
                           k=int(k), fval=float(out["fval"]),
                           sha256=dict(A=sha(A), b=sha(b), x0=sha(x0), u=sha(u)))
        print("%-44s k=%5d fval=%.12e" % (name, k, float(out["fval"])))
    with open(os.path.join(HERE, "index.json"), "w") as fh:
        json.dump(index, fh, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
