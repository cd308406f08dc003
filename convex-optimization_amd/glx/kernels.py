"""Single-kernel entry points of libglx (``glx_residual`` / ``glx_gradient`` / ``glx_prox`` /
``glx_residual_gradient``).

These are the dense products and the group prox of the reference iteration exposed one at a
time — ``A @ x - b`` (gl_ProxGD_primal.py:25,61), ``A.T @ r`` (:129) and ``prox_th``
(:65-71) — used by the kernel-level tests and available for composition. All tensors are
contiguous device tensors of one dtype (float32 / float64).
"""
from __future__ import annotations

import ctypes
from typing import Tuple

import torch

from . import _lib
from ._lib import check, lib


def _dt(t: torch.Tensor) -> int:
    if t.dtype == torch.float64:
        return _lib.GLX_F64
    if t.dtype == torch.float32:
        return _lib.GLX_F32
    raise ValueError("float32 or float64 required")


def _ws(dtype: int, m: int, n: int, l: int, device) -> torch.Tensor:
    nb = ctypes.c_size_t(0)
    check(lib().glx_kernel_workspace_bytes(dtype, m, n, l, ctypes.byref(nb)))
    return torch.empty(int(nb.value), dtype=torch.uint8, device=device)


def _stream(device) -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def residual(A: torch.Tensor, X: torch.Tensor, B: torch.Tensor, variant: int = 0
             ) -> Tuple[torch.Tensor, torch.Tensor]:
    """R = A X - B and 1/2 ||R||_F^2 (a 1-element float64 device tensor)."""
    m, n = A.shape
    l = X.shape[1]
    dt = _dt(A)
    R = torch.empty((m, l), dtype=A.dtype, device=A.device)
    h = torch.empty(1, dtype=torch.float64, device=A.device)
    ws = _ws(dt, m, n, l, A.device)
    check(lib().glx_residual(dt, m, n, l, A.data_ptr(), X.data_ptr(), B.data_ptr(), R.data_ptr(),
                             h.data_ptr(), ws.data_ptr(), ws.numel(), variant, _stream(A.device)))
    return R, h


def residual_batch(A: torch.Tensor, Xs, B: torch.Tensor, variant: int = 0):
    """R_i = A X_i - B for up to three right-hand sides in one pass over A; also returns the
    squared norms ||R_i||^2 (float64 device tensor)."""
    m, n = A.shape
    l = Xs[0].shape[1]
    dt = _dt(A)
    Rs = [torch.empty((m, l), dtype=A.dtype, device=A.device) for _ in Xs]
    sq = torch.empty(4, dtype=torch.float64, device=A.device)
    ws = _ws(dt, m, n, l, A.device)
    xp = (ctypes.c_void_p * 3)(*[x.data_ptr() for x in Xs], *([None] * (3 - len(Xs))))
    rp = (ctypes.c_void_p * 3)(*[r.data_ptr() for r in Rs], *([None] * (3 - len(Rs))))
    check(lib().glx_residual_batch(dt, m, n, l, A.data_ptr(), len(Xs), xp, B.data_ptr(), rp,
                                   sq.data_ptr(), ws.data_ptr(), ws.numel(), variant,
                                   _stream(A.device)))
    return Rs, sq


def gradient(A: torch.Tensor, R: torch.Tensor) -> torch.Tensor:
    """G = A^T R."""
    m, n = A.shape
    l = R.shape[1]
    dt = _dt(A)
    G = torch.empty((n, l), dtype=A.dtype, device=A.device)
    ws = _ws(dt, m, n, l, A.device)
    check(lib().glx_gradient(dt, m, n, l, A.data_ptr(), R.data_ptr(), G.data_ptr(), ws.data_ptr(),
                             ws.numel(), _stream(A.device)))
    return G


def residual_gradient(A: torch.Tensor, X: torch.Tensor, B: torch.Tensor, one_pass: bool = False
                      ) -> Tuple[torch.Tensor, torch.Tensor, bool]:
    """R = A X - B and G = A^T R: two passes over A (the faster path), or with one_pass=True
    the fused kernel that reads A from HBM once, where the shape and device allow it.
    Returns (R, G, one_pass_ran)."""
    m, n = A.shape
    l = X.shape[1]
    dt = _dt(A)
    R = torch.empty((m, l), dtype=A.dtype, device=A.device)
    G = torch.empty((n, l), dtype=A.dtype, device=A.device)
    ws = _ws(dt, m, n, l, A.device)
    fused = ctypes.c_int(0)
    check(lib().glx_residual_gradient(dt, m, n, l, A.data_ptr(), X.data_ptr(), B.data_ptr(),
                                      R.data_ptr(), G.data_ptr(), ws.data_ptr(), ws.numel(),
                                      1 if one_pass else 0, ctypes.byref(fused), _stream(A.device)))
    return R, G, bool(fused.value)


def residual_gradient2(A: torch.Tensor, X0: torch.Tensor, X1: torch.Tensor, B: torch.Tensor,
                       one_pass: bool = True
                       ) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor, bool]:
    """The line-search trial's batch and the next gradient: R0 = A X0 - B, R1 = A X1 - B and
    G = A^T R1, with one read of A (the l = 16 role-split kernel) where the shape and device
    allow it, else A @ [X0 | X1] then A^T R1. Returns (R0, R1, G, one_pass_ran)."""
    m, n = A.shape
    l = X0.shape[1]
    dt = _dt(A)
    R0 = torch.empty((m, l), dtype=A.dtype, device=A.device)
    R1 = torch.empty((m, l), dtype=A.dtype, device=A.device)
    G = torch.empty((n, l), dtype=A.dtype, device=A.device)
    ws = _ws(dt, m, n, l, A.device)
    ran = ctypes.c_int(0)
    check(lib().glx_residual_gradient2(dt, m, n, l, A.data_ptr(), X0.data_ptr(), X1.data_ptr(),
                                       B.data_ptr(), R0.data_ptr(), R1.data_ptr(), G.data_ptr(),
                                       ws.data_ptr(), ws.numel(), 1 if one_pass else 0,
                                       ctypes.byref(ran), _stream(A.device)))
    return R0, R1, G, bool(ran.value)


def flagged_rows_product(At: torch.Tensor, E: torch.Tensor, row_masks: torch.Tensor,
                         form: int = 0) -> torch.Tensor:
    """Y = sum over the rows k with row_masks[k] != 0 of At[k]^T E[k] (m x l): the split-candidate
    trial's A e from the transposed copy At = A^T (n x m). form 0: the MFMA row form
    (m % 64 == 0), 1: the VALU column-list gather of rounds 2-4, 2: the bitmap gather (the
    solver's default; 1 and 2 need bit c of row_masks[k] == (E[k][c] != 0)). row_masks: int32
    device tensor of n (+ padding) column masks."""
    n, m = At.shape
    l = E.shape[1]
    dt = _dt(At)
    Y = torch.empty((m, l), dtype=At.dtype, device=At.device)
    ws = _ws(dt, m, n, l, At.device)
    check(lib().glx_flagged_rows_product(dt, m, n, l, At.data_ptr(), E.data_ptr(),
                                         row_masks.data_ptr(), Y.data_ptr(), int(form),
                                         ws.data_ptr(), ws.numel(), _stream(At.device)))
    return Y


def prox(W: torch.Tensor, t: float, mu: float, thres: float = 1e-3
         ) -> Tuple[torch.Tensor, torch.Tensor]:
    """Group prox with the reference's denominator quirk; returns (X, [sum ||x_i||, max|x|])."""
    n, l = W.shape
    dt = _dt(W)
    X = torch.empty_like(W)
    sums = torch.empty(2, dtype=torch.float64, device=W.device)
    ws = _ws(dt, 1, n, l, W.device)
    check(lib().glx_prox(dt, n, l, W.data_ptr(), float(t), float(mu), float(thres), X.data_ptr(),
                         sums.data_ptr(), ws.data_ptr(), ws.numel(), _stream(W.device)))
    return X, sums
