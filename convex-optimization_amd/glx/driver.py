"""The reference's demo driver (``code/main.py``) on the MI355X solvers.

Same instance, the same solver loop, the same per-solver log line and the same Markdown
"Statistics" table as ``main.py``, so a run reads like the reference's report
(``doc/report.md:439-447``):

- ``gen_data`` follows ``main.py:37-51``: MT19937 seed 97006855, (m, n, l) = (256, 512, 2),
  mu = 1e-2, 10% row support.
- ``solve_routine`` follows ``main.py:113-130``: one log line ``[mode      ]: cpu: …, iter: …``
  with the same keys and number formats.
- ``write_to_table`` follows ``main.py:94-110``: a Markdown table titled "Statistics".
- The solver registry and option dicts follow ``main.py:169-197``, for the five primal gradient
  methods this build implements (GD, FGD, SGD, ProxGD, FProxGD).

Differences, all forced by what the image lacks:
- The two ``err-to-cvx-*`` columns (``main.py:122-123``) become one ``err-to-x*`` column.
  x* is a high-accuracy minimiser loaded from ``--xstar``
  (``tests/golden/default_xstar.npz`` for the default instance, made by
  ``tests/golden/make_xstar.py``). It reproduces the report's CVX-Mosek row. Without
  ``--xstar`` the column reads ``n/a``. cvxpy, Mosek and Gurobi are not installed.
- The svg plots (``main.py:200-235``) are replaced by ``f_hist.npz`` in ``--dest_dir``: the
  per-solver objective histories and f* = obj(u) those plots are drawn from. matplotlib is
  not installed.
- The ALM/ADMM solvers are out of scope.

Every solver runs on the GPU through libglx (``glx.solver.solve``); there is no CPU path.

    PYTHONPATH=convex-optimization_amd python -m glx.driver --xstar tests/golden/default_xstar.npz
"""
from __future__ import annotations

import argparse
import logging
import os
import sys
from typing import Any, Callable, Dict, Optional, TextIO

import numpy as np

LOGGER = "opt"
SEED = 97006855


def gen_data(seed: int = SEED, m: int = 256, n: int = 512, l: int = 2, mu: float = 1e-2):
    """main.py:37-51: A, b = A u, u with round(0.1 n) nonzero rows, x0 ~ N(0, 1).

    Returns (n, m, l, mu, A, b, u, x0, errfun, errfun_exact, sparsity), in main.py's order.
    """
    g = np.random.Generator(np.random.MT19937(seed=seed))
    A = g.standard_normal(size=(m, n))
    k = round(n * 0.1)
    support = g.permutation(n)[:k]
    u = np.zeros((n, l))
    u[support, :] = g.standard_normal(size=(k, l))
    b = A @ u
    x0 = g.standard_normal(size=(n, l))

    def errfun(x1, x2):                          # main.py:48
        return np.linalg.norm(x1 - x2, "fro") / (1 + np.linalg.norm(x1, "fro"))

    def errfun_exact(x):                         # main.py:49
        return np.linalg.norm(x - u, "fro") / (1 + np.linalg.norm(x, "fro"))

    def sparsity(x):                             # main.py:50
        return np.sum(np.abs(x) > 1e-6 * np.max(np.abs(x))) / (n * l)

    return n, m, l, mu, A, b, u, x0, errfun, errfun_exact, sparsity


def obj_func(A, b, mu, x) -> float:
    """main.py:30-34 (the objective at mu, used for f* = obj(u) in the relative-objective plot)."""
    r = A @ x - b
    return 0.5 * float(np.sum(r * r)) + mu * float(np.linalg.norm(x, axis=1).sum())


def _glx_solvers() -> Dict[str, Callable]:
    """main.py:169-182, restricted to the methods this build implements, in main.py's order."""
    from glx.solver import solve

    def bind(name):
        def f(x0, A, b, mu, opts):
            return solve(name, x0, A, b, mu, opts)
        f.__name__ = name
        return f

    return {
        "SGD Primal": bind("gl_SGD_primal"),
        "GD Primal": bind("gl_GD_primal"),
        "FGD Primal": bind("gl_FGD_primal"),
        "ProxGD Primal": bind("gl_ProxGD_primal"),
        "FProxGD Primal": bind("gl_FProxGD_primal"),
    }


def solve_routine(mode: str, func: Callable, x0, A, b, mu, opts, errfun, errfun_exact, sparsity,
                  xstar: Optional[np.ndarray] = None):
    """main.py:113-130. Returns (x, num_iters, out, log_dict) and logs one line."""
    x, num_iters, out = func(x0, A, b, mu, opts)
    x = np.asarray(x.cpu().numpy() if hasattr(x, "cpu") else x)
    log_dict = {
        "cpu": "%5.2f" % out["tt"],
        "iter": "%5d" % (-1 if num_iters is None else num_iters),
        "optval": "%6.5E" % out["fval"],
        "sparsity": "%6.4f" % sparsity(x),
        "err-to-exact": "%3.2E" % errfun_exact(x),
        "err-to-x*": "n/a" if xstar is None else "%3.2E" % errfun(xstar, x),
    }
    line = ("[%-10s]: " % mode) + ", ".join(k + ": " + v for k, v in log_dict.items())
    logging.getLogger(LOGGER).info(line)
    return x, num_iters, out, log_dict


def write_to_table(log_dicts: Dict[str, Dict[str, str]], stream: TextIO = sys.stdout) -> str:
    """main.py:94-110: a Markdown table "Statistics", one row per solver, strings left-aligned."""
    headers = None
    rows = []
    for mode, d in log_dicts.items():
        if headers is None:
            headers = ["solver"] + list(d.keys())
        rows.append([mode] + [v.strip() for v in d.values()])
    assert headers is not None, "no solver ran"
    w = [max(len(h), *(len(r[i]) for r in rows)) for i, h in enumerate(headers)]
    fmt = lambda cells: "|" + "|".join(" %-*s " % (w[i], c) for i, c in enumerate(cells)) + "|"
    text = "\n".join(["# Statistics", fmt(headers),
                      "|" + "|".join("-" * (wi + 2) for wi in w) + "|"] + [fmt(r) for r in rows])
    stream.write(text + "\n")
    return text


def setup_logger(log_file: Optional[str], level=logging.INFO) -> logging.Logger:
    """main.py:54-64: the same formatter, to the log file (append) and to stderr."""
    log = logging.getLogger(LOGGER)
    log.setLevel(level)
    log.handlers.clear()
    fmt = logging.Formatter("%(asctime)s: %(levelname)-5s %(message)s")
    handlers = [logging.StreamHandler()]
    if log_file:
        handlers.append(logging.FileHandler(log_file, mode="a"))
    for h in handlers:
        h.setFormatter(fmt)
        log.addHandler(h)
    return log


def run(solvers: Optional[Dict[str, Callable]] = None, solvers_opts: Optional[Dict[str, dict]] = None,
        xstar: Optional[np.ndarray] = None, dest_dir: Optional[str] = None, seed: int = SEED,
        size=(256, 512, 2), stream: TextIO = sys.stdout) -> Dict[str, Any]:
    """The body of main.py's __main__ block (main.py:141-235) without the CVX solvers and plots.

    ``solvers`` defaults to the GPU solvers; tests pass other callables with the same signature.
    Returns {"log_dicts", "f_hists", "f_star", "xs"}.
    """
    m, n, l = size
    n, m, l, mu, A, b, u, x0, errfun, errfun_exact, sparsity = gen_data(seed, m, n, l)
    if xstar is not None and np.shape(xstar) != (n, l):
        raise ValueError(f"x* has shape {np.shape(xstar)}, the instance needs {(n, l)}")
    solvers = _glx_solvers() if solvers is None else solvers
    solvers_opts = solvers_opts or {}
    log_dicts, f_hists, xs = {}, {}, {}
    for mode, solver in solvers.items():             # main.py:199-205
        x, _, out, log_dict = solve_routine(mode, solver, x0, A, b, mu, dict(solvers_opts.get(mode, {})),
                                            errfun, errfun_exact, sparsity, xstar)
        if "f_hist" in out:
            f_hists[mode] = np.asarray(out["f_hist"], dtype=np.float64)
        log_dicts[mode] = log_dict
        xs[mode] = x
    write_to_table(log_dicts, stream)
    f_star = obj_func(A, b, mu, u)
    if dest_dir:
        os.makedirs(dest_dir, exist_ok=True)
        np.savez(os.path.join(dest_dir, "f_hist.npz"), f_star=f_star,
                 **{k.replace(" ", "_"): v for k, v in f_hists.items()})
    return {"log_dicts": log_dicts, "f_hists": f_hists, "f_star": f_star, "xs": xs}


def main(argv=None) -> int:
    p = argparse.ArgumentParser(
        formatter_class=argparse.ArgumentDefaultsHelpFormatter,
        description=r"A demo that solves the optimization problem "
                    r"$\min_x{0.5 * ||A * x - b||_2^2 + mu * ||x||_{1,2}}$ on the GPU")
    p.add_argument("--log", default="opt.log", help="Path to the logging file.")
    p.add_argument("--dest_dir", default="figures", help="Destination directory.")
    p.add_argument("--xstar", default=None, help="npz with the reference minimiser x (err-to-x* column).")
    p.add_argument("--seed", type=int, default=SEED)
    p.add_argument("--size", default="256,512,2", help="m,n,l")
    p.add_argument("--solvers", default=None, help="comma-separated subset, e.g. 'ProxGD Primal'")
    a = p.parse_args(argv)
    setup_logger(a.log)
    size = tuple(int(v) for v in a.size.split(","))
    xstar = np.load(a.xstar)["x"] if a.xstar else None
    solvers = _glx_solvers()
    if a.solvers:
        keep = [s.strip() for s in a.solvers.split(",")]
        unknown = [s for s in keep if s not in solvers]
        if unknown:
            p.error(f"unknown solver(s) {unknown}; choose from {list(solvers)}")
        solvers = {k: solvers[k] for k in keep}
    run(solvers, xstar=xstar, dest_dir=a.dest_dir, seed=a.seed, size=size)
    return 0


if __name__ == "__main__":
    sys.exit(main())
