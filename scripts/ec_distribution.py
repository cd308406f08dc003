"""The split-candidate e / e_c over whole NS solves (round 5): per trial
batch, FProxGD's e_c flagged rows (GLX_GATHER=rows) and nonzeros (GLX_GATHER=valu) with the nnz
budget off (every batch gathered), and ProxGD's e rows, through glx_session_split_trace. One JSON
line per (method, form): quantiles, per-500-iteration means, whole-solve it/s and the gather's
kernel time (events on every 4th launch)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "convex-optimization_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    m, n, l = 8192, 16384, 32
    dev = torch.device("cuda", 0)
    A, b, x0, info = bench.reference_instance("gl_FProxGD_primal", "f64", m, n, l, 0, m,
                                              torch.float64, dev)
    mu = 1e-2
    opts = {"alpha0": 1.0 / (m ** 0.5 + n ** 0.5) ** 2, "profile": 4}
    from glx.solver import Session
    cases = [("gl_FProxGD_primal", "rows", "10"), ("gl_FProxGD_primal", "bm", "10"),
             ("gl_FProxGD_primal", "rows", None), ("gl_FProxGD_primal", "bm", None),
             ("gl_ProxGD_primal", "rows", None), ("gl_ProxGD_primal", "bm", None),
             ("gl_ProxGD_primal", "lists", None)]
    for method, form, budget in cases:
        os.environ["GLX_GATHER"] = form
        if budget is None:
            os.environ.pop("GLX_SPLIT_NNZ", None)
        else:
            os.environ["GLX_SPLIT_NNZ"] = budget
        x = x0.clone()
        s = Session(method, x, A, b, mu, dict(opts))
        s.run(0)
        tr = s.split_trace()
        gn, gms = s.kernel_time(2)
        an, ams = s.kernel_time(0)
        res = s.finish()
        s.close()
        g = tr[tr >= 0]
        chunks = [float(np.mean(c[c >= 0])) if np.any(c >= 0) else -1.0
                  for c in np.array_split(tr, max(1, len(tr) // 500))]
        print(json.dumps({"method": method, "form": form, "budget": budget, "k": res["k"],
                          "it_s": res["k"] / res["tt"], "batches": int(len(tr)),
                          "gathered": int(len(g)), "dense": int(np.sum(tr < 0)),
                          "frac_n_q": [float(np.quantile(g, q) / n) for q in (0.1, 0.5, 0.9, 0.99)]
                          if len(g) else None,
                          "mean_frac_n_per_500": [round(c / n, 4) for c in chunks],
                          "gather_us": 1e3 * gms / gn if gn else None,
                          "ax_us": 1e3 * ams / an if an else None}), flush=True)


if __name__ == "__main__":
    main()
