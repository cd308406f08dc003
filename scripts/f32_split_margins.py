"""fp32 FProxGD: the dense [xc | y_next] batch against the split-candidate batch (A y_next by
linearity, GLX_SPLIT_F32=1) — fval / f_hist drift against the reference's fp32 golden runs and
the oracle (fp32 NumPy) on larger instances. Prints one JSON line per (case, mode)."""
import json
import os
import sys
import warnings

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "convex-optimization_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

from conftest import golden_case, golden_inputs  # noqa: E402
from oracle import numpy_ref  # noqa: E402


def rel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    n = min(len(a), len(b)) if a.ndim else None
    if n is not None:
        a, b = a[:n], b[:n]
    return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-300)))


def run(A, b, x0, mu, opts, mode):
    from gl_FProxGD_primal import gl_FProxGD_primal
    if mode == "split":
        os.environ["GLX_SPLIT_F32"] = "1"
        os.environ["GLX_SPLIT_CAND"] = "1"
    else:
        os.environ.pop("GLX_SPLIT_F32", None)
        os.environ.pop("GLX_SPLIT_CAND", None)
    return gl_FProxGD_primal(x0, A, b, mu, dict(opts))


def main():
    cases = []
    for name in ("mid_256x512x32_f32_gl_FProxGD_primal", "mid_384x640x16_f32_gl_FProxGD_primal"):
        meta, gold = golden_case(name)
        A, b, u, x0, mu = golden_inputs(meta)
        cases.append((name, A, b, x0, mu, dict(meta["opts"]), int(gold["k"]), gold["fval"], gold["f_hist"]))
    big = [(2048, 4096, 32, 2024, 3), (1024, 2048, 16, 7, 40), (2048, 4096, 16, 11, 60)]
    if "--c3" in sys.argv:
        big.append((8192, 16384, 32, 97006855, 2))
    for m, n, l, seed, maxit in big:
        A, b, u, x0, mu = numpy_ref.gen_data(m, n, l, seed)
        A, b, x0 = (a.astype(np.float32) for a in (A, b, x0))
        opts = {"alpha0": numpy_ref.step_size_for(m, n), "maxit": maxit}
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            xr, kr, outr = numpy_ref.gl_FProxGD_primal(x0, A, b, mu, dict(opts))
        cases.append(("oracle_%dx%dx%d_it%d" % (m, n, l, maxit), A, b, x0, mu, opts, kr, outr["fval"],
                      np.asarray(outr["f_hist"], float)))
    for name, A, b, x0, mu, opts, kg, fg, fhg in cases:
        for mode in ("dense", "split"):
            x, k, out = run(A, b, x0, mu, opts, mode)
            print(json.dumps({"case": name, "mode": mode, "k": k, "k_ref": kg,
                              "fval_rel": rel(out["fval"], fg),
                              "fhist_rel": rel(np.asarray(out["f_hist"], float), fhg)}), flush=True)


if __name__ == "__main__":
    main()
