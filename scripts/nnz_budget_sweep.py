"""Whole-solve FProxGD throughput against the split-candidate nnz budget (GLX_SPLIT_NNZ, a
fraction of n above which a gathered batch trips to kFistaDenseRun dense batches): C3 (fp32,
GLX_SPLIT_F32=1 with the f32 LDS-DMA tile) and NS fp64. One JSON line per (case, budget) with tt,
k, fval and the batch statistics (glx_result.stats[3..6]: gathered / dense batches, summed
nnz(e_c), A thr(x_k) restores)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "convex-optimization_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def whole(method, A, b, x0, mu, opts):
    from glx.solver import Session
    x = x0.clone()
    s = Session(method, x, A, b, mu, dict(opts))
    try:
        s.run(0)
        return s.finish()
    finally:
        s.close()


def main():
    m, n, l = 8192, 16384, 32
    budgets = [float(v) for v in (sys.argv[1:] or ["0.35", "0.5", "0.65"])]
    for dtype, label in ((torch.float32, "C3_f32"), (torch.float64, "NS_f64")):
        A, b, x0 = bench.make_instance(m, n, l, 0, m, dtype, "cuda")
        mu = 1e-2
        opts = {"alpha0": 1.0 / (m ** 0.5 + n ** 0.5) ** 2}
        runs = [("dense", None)] + [("split", bv) for bv in budgets]
        for mode, bv in runs:
            if dtype == torch.float32:
                os.environ["GLX_AX_DMA32"] = "1"
                if mode == "split":
                    os.environ["GLX_SPLIT_F32"] = "1"
                else:
                    os.environ.pop("GLX_SPLIT_F32", None)
            os.environ["GLX_SPLIT_FISTA"] = "1" if mode == "split" else "0"
            if bv is not None:
                os.environ["GLX_SPLIT_NNZ"] = str(bv)
            whole("gl_FProxGD_primal", A, b, x0, mu, opts)   # warm
            r = whole("gl_FProxGD_primal", A, b, x0, mu, opts)
            st = r["stats"]
            print(json.dumps({"case": label, "mode": mode, "budget": bv, "k": r["k"], "tt": r["tt"],
                              "it_s": r["k"] / r["tt"], "fval": float(r["fval"]),
                              "gathered": st[3], "dense": st[4],
                              "mean_nnz_frac": (st[5] / st[3] / n) if st[3] else None,
                              "restores": st[6]}), flush=True)
        del A, b, x0
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
