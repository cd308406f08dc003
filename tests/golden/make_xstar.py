"""Generate tests/golden/default_xstar.npz: a high-accuracy minimiser x* of the default instance.

main.py reports each solver's distance to the CVX-Mosek and CVX-Gurobi solutions
(``main.py:121-123``, ``errfun`` at ``main.py:48``). cvxpy and the commercial back-ends are not
in this image, so the driver (``glx/driver.py``) reports the distance to this fixture instead.

x* minimises 0.5||Ax-b||_F^2 + mu * sum_i ||x_i||_2 on main.py's default instance
(``gen_data``, ``main.py:37-51``; restated in ``oracle.numpy_ref.gen_data``). It is computed here
with plain NumPy in two stages: accelerated proximal gradient (FISTA with adaptive restart, step
1/L with L = ||A||_2^2, exact group soft-threshold) until the support is identified, then
Newton's method on the support's stationarity equations
A_S^T (A_S x_S - b) + mu x_i / ||x_i|| = 0 (smooth there). The result must have a proximal
fixed-point residual ||x - prox(x - grad/L)|| * L below 1e-11 (rounding level at L ~ 1.5e3), which also certifies the rows
off the support (||A_i^T r|| <= mu). The residual is stored with x* so the fixture documents its
own accuracy.

    python tests/golden/make_xstar.py
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle.numpy_ref import gen_data  # noqa: E402


def group_shrink(w, tau):
    nrm = np.linalg.norm(w, axis=1, keepdims=True)
    scale = np.where(nrm > tau, 1.0 - tau / np.where(nrm > 0, nrm, 1.0), 0.0)
    return w * scale


def objective(A, b, x, mu):
    r = A @ x - b
    return 0.5 * float(np.sum(r * r)) + mu * float(np.linalg.norm(x, axis=1).sum())


def fixed_point_residual(A, b, x, mu, L):
    g = A.T @ (A @ x - b)
    return float(np.linalg.norm(x - group_shrink(x - g / L, mu / L)) * L)


def newton_on_support(A, b, x, mu, iters=30):
    S = np.flatnonzero(np.linalg.norm(x, axis=1) > 0)
    l = x.shape[1]
    AS = A[:, S]
    H = np.kron(AS.T @ AS, np.eye(l))
    Atb = AS.T @ b
    xs = x[S].copy()
    for _ in range(iters):
        nrm = np.linalg.norm(xs, axis=1, keepdims=True)
        F = AS.T @ (AS @ xs) - Atb + mu * xs / nrm
        J = H.copy()
        for k in range(len(S)):
            v = xs[k:k + 1].T
            blk = mu * (np.eye(l) / nrm[k, 0] - (v @ v.T) / nrm[k, 0] ** 3)
            J[k * l:(k + 1) * l, k * l:(k + 1) * l] += blk
        step = np.linalg.solve(J, F.reshape(-1)).reshape(xs.shape)
        xs -= step
        if np.abs(step).max() < 1e-16:
            break
    out = np.zeros_like(x)
    out[S] = xs
    return out


def solve(A, b, mu, tol=1e-7, maxit=200000):
    L = float(np.linalg.norm(A, 2)) ** 2
    x = np.zeros((A.shape[1], b.shape[1]))
    y, theta, f_prev = x.copy(), 1.0, np.inf
    for it in range(maxit):
        if it % 100 == 0 and fixed_point_residual(A, b, x, mu, L) < tol:
            break
        xn = group_shrink(y - (A.T @ (A @ y - b)) / L, mu / L)
        f = objective(A, b, xn, mu)
        if f > f_prev:                      # adaptive restart (O'Donoghue & Candes)
            y, theta = x.copy(), 1.0
            continue
        th = 0.5 * (1.0 + np.sqrt(1.0 + 4.0 * theta * theta))
        y = xn + ((theta - 1.0) / th) * (xn - x)
        x, theta, f_prev = xn, th, f
    x = newton_on_support(A, b, x, mu)
    return x, fixed_point_residual(A, b, x, mu, L), it + 1


def main():
    A, b, u, x0, mu = gen_data()
    x, res, iters = solve(A, b, mu)
    f = objective(A, b, x, mu)
    print(f"x*: fval {f:.15e}  fixed-point residual {res:.3e}  iterations {iters}")
    assert res < 1e-11, res
    np.savez_compressed(os.path.join(HERE, "default_xstar.npz"), x=x, fval=f, residual=res,
                        mu=mu, seed=97006855)


if __name__ == "__main__":
    main()
