"""Measure the fp32 parity margins (relative fval error, k) of the HIP solvers against the
reference's golden fp32 runs and the fp32 oracle at larger sizes. Prints one JSON line per case.

    python scripts/fp32_parity_probe.py
"""
import importlib
import json
import os
import sys
import warnings

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "convex-optimization_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402

from conftest import golden_case, golden_index, golden_inputs  # noqa: E402
from oracle import numpy_ref  # noqa: E402


def rel(a, b):
    return abs(float(a) - float(b)) / abs(float(b))


def main():
    for name in sorted(golden_index()):
        meta, gold = golden_case(name)
        if meta["dtype"] != "f32":
            continue
        A, b, u, x0, mu = golden_inputs(meta)
        mod = importlib.import_module(meta["solver"])
        x, k, out = getattr(mod, meta["solver"])(x0, A, b, mu, dict(meta["opts"]))
        fh = np.asarray(out["f_hist"], float)
        gf = np.asarray(gold["f_hist"], float)
        n = min(len(fh), len(gf))
        print(json.dumps({"case": name, "k": k, "gold_k": int(gold["k"]), "rel_fval": rel(out["fval"], gold["fval"]),
                          "max_rel_fhist_common": float(np.max(np.abs(fh[:n] - gf[:n]) / np.abs(gf[:n]))),
                          "gold_fval": float(gold["fval"])}), flush=True)
    for solver, shape, maxit in [("gl_FProxGD_primal", (8192, 16384, 32), 2), ("gl_FProxGD_primal", (2048, 4096, 32), 40),
                                 ("gl_ProxGD_primal", (2048, 4096, 32), 40)]:
        m, n, l = shape
        A, b, u, x0, mu = numpy_ref.gen_data(m, n, l, 97006855)
        A, b, x0 = (a.astype(np.float32) for a in (A, b, x0))
        opts = {"alpha0": numpy_ref.step_size_for(m, n), "maxit": maxit}
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            xr, kr, outr = numpy_ref.SOLVERS[solver](x0, A, b, mu, dict(opts))
        x, k, out = getattr(importlib.import_module(solver), solver)(x0, A, b, mu, dict(opts))
        fh = np.asarray(out["f_hist"], float)
        fo = np.asarray(outr["f_hist"], float)
        n_ = min(len(fh), len(fo))
        print(json.dumps({"case": "%s_f32_%dx%dx%d_maxit%d" % (solver, m, n, l, maxit), "k": k, "oracle_k": kr,
                          "rel_fval": rel(out["fval"], outr["fval"]),
                          "max_rel_fhist": float(np.max(np.abs(fh[:n_] - fo[:n_]) / np.abs(fo[:n_])))}), flush=True)


if __name__ == "__main__":
    main()
