"""Host side of the drop-in boundary: ``gl_<method>(x0, A, b, mu_0, opts) -> (x, iters, out)``.

Mirrors the reference's solver interface (``code/gl_ProxGD_primal.py:9`` and siblings):

* ``opts`` is merged over the per-method defaults exactly like ``{**default_opts, **opts}``
  (``gl_ProxGD_primal.py:21``): unknown keys are ignored, the caller's dict is not mutated.
* ``x0`` is copied (``:49``); ``A`` and ``b`` are read-only.
* returns ``(x, k, out)`` with ``out = {"tt", "fval", "f_hist", "f_hist_best"}`` (``:139-146``);
  ``x`` comes back as the caller's array type (NumPy in → NumPy out, torch in → torch out).
* an unsupported ``step_type`` raises ``ValueError`` (the reference logs an error and then
  fails on ``None``, ``:100-101``).

Everything numeric runs in libglx (HIP kernels + the native iteration driver); PyTorch only
provides device memory, the stream and the multi-process bootstrap. There is no CPU path.

Build-only option keys (ignored by the reference): ``exact_objective`` (ProxGD: recompute
A@x for every objective instead of reusing the accepted trial residual), ``profile``,
``max_total_iters``, ``ax_variant``, ``split_cand`` (0 auto, 1 on, 2 off), ``dc_window``
(device-controlled line search: 0 auto, -1 off, k iterations in flight), ``shard_rows``
(ProxGD with a communicator: 0 auto = the row-sharded schedule, 1 on, 2 off = the gradient
all-reduce schedule), ``shard_model`` (bench.py only: the per-rank timing model of G ranks at
world size 1; ``solve`` refuses it), ``device``, ``comm``.
"""
from __future__ import annotations

import ctypes
import logging
from typing import Any, Dict, List, Optional, Tuple

import numpy as np
import torch

from . import _lib
from ._lib import GlxOpts, GlxProblem, GlxResult, check, lib

logger = logging.getLogger("opt")

_REF_KEYS = {
    "maxit": "maxit", "thres": "thres", "alpha0": "alpha0", "ftol": "ftol",
    "stable_len_threshold": "stable_len_threshold",
    "line_search_attenuation_coeffi": "ls_coeff", "maxit_line_search_iter": "ls_maxit",
    "delta": "delta",
}
_BUILD_KEYS = {"exact_objective", "profile", "max_total_iters", "ax_variant", "split_cand",
               "dc_window", "shard_rows", "shard_model"}


def _device(opts: Dict[str, Any]) -> torch.device:
    if not torch.cuda.is_available():
        raise RuntimeError("glx runs on an AMD Instinct GPU (HIP); no GPU is visible and there is "
                           "no CPU fallback")
    dev = opts.get("device")
    if dev is None:
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device(dev)


def make_opts(method: int, opts: Dict[str, Any]) -> GlxOpts:
    """Per-method defaults (``gl_*_primal.py`` default_opts) overridden by ``opts``."""
    o = _lib.default_opts(method)
    for key, field in _REF_KEYS.items():
        if key in opts:
            setattr(o, field, type(getattr(o, field))(opts[key]))
    if "step_type" in opts:
        st = opts["step_type"]
        if st not in _lib.STEP_TYPES:
            raise ValueError("Unsupported type: %r" % (st,))
        if method in (_lib.GLX_SGD, _lib.GLX_GD) and st == "line_search":
            raise ValueError("Unsupported type: 'line_search' (SGD/GD have no line search)")
        o.step_type = _lib.STEP_TYPES[st]
    for key in _BUILD_KEYS:
        if key in opts:
            setattr(o, key, int(opts[key]))
    return o


def _as_device(a, device, dtype) -> torch.Tensor:
    t = torch.as_tensor(a).to(device=device, dtype=dtype).contiguous()
    if t.data_ptr() % 16:   # e.g. a view A[1:] with odd n: libglx needs 16-byte aligned rows
        t = t.clone()
    return t


def _dtype_of(A) -> torch.dtype:
    dt = A.dtype if isinstance(A, torch.Tensor) else torch.from_numpy(np.empty(0, dtype=np.asarray(A).dtype)).dtype
    return torch.float32 if dt == torch.float32 else torch.float64


def workspace(problem: GlxProblem, o: GlxOpts, device) -> torch.Tensor:
    nbytes = ctypes.c_size_t(0)
    check(lib().glx_workspace_bytes(ctypes.byref(problem), ctypes.byref(o), ctypes.byref(nbytes)))
    return torch.empty(int(nbytes.value), dtype=torch.uint8, device=device)


def _lambda_max(A: torch.Tensor, comm=None, max_steps: int = 400) -> float:
    """``np.max(LA.eigvals(A.T @ A))`` (gl_SGD_primal.py:35-37, gl_GD_primal.py:43-45) for the
    optional continuous_subgradient_flag, without forming the n x n Gram matrix and without a
    library eigensolver on the device: Lanczos on the operator v -> A^T (A v), whose two products
    are libglx's own kernels (glx_residual with b = 0, glx_gradient; with row-sharded A the
    product is all-reduced over the ranks, so every rank runs the same recurrence). The
    recurrence and its full re-orthogonalisation run on the host in float64 on n-vectors; the
    largest eigenvalue of the k x k tridiagonal matrix is taken once its Ritz residual
    beta_k |s_k| is below 1e-13 of it (the eigenvalue itself is then accurate to ~1e-16 relative),
    or when the Krylov space is all of R^n (k = n: exact). A fixed start vector (seeded), so the
    result is the same on every rank and from run to run."""
    import numpy as np
    from . import kernels
    a = A if A.dtype == torch.float64 else A.to(torch.float64)
    m, n = a.shape
    zero = torch.zeros((m, 1), dtype=torch.float64, device=a.device)
    rng = np.random.default_rng(20240611)
    q = rng.standard_normal(n)
    q /= np.linalg.norm(q)
    Q = np.zeros((min(n, max_steps) + 1, n))
    alphas, betas = [], []
    q_prev, beta = np.zeros(n), 0.0
    theta = 0.0
    for k in range(min(n, max_steps)):
        Q[k] = q
        r, _ = kernels.residual(a, torch.from_numpy(np.ascontiguousarray(q[:, None])).to(a.device), zero)   # A q
        w_t = kernels.gradient(a, r)                                                   # A^T A q
        if comm is not None:
            comm.allreduce_(w_t)
        w = w_t[:, 0].cpu().numpy()
        alpha = float(q @ w)
        w = w - alpha * q - beta * q_prev
        for _ in range(2):   # full re-orthogonalisation against the basis so far
            w -= Q[:k + 1].T @ (Q[:k + 1] @ w)
        alphas.append(alpha)
        beta = float(np.linalg.norm(w))
        T = np.diag(alphas) + np.diag(betas, 1) + np.diag(betas, -1)
        ev, evec = np.linalg.eigh(T)
        theta = float(ev[-1])
        # an invariant subspace (beta ~ 0), or the Ritz pair of theta converged
        if beta <= 1e-14 * abs(theta) or (k >= 4 and abs(beta * evec[-1, -1]) <= 1e-13 * abs(theta)):
            break
        betas.append(beta)
        q_prev, q = q, w / beta
    return theta


def _replay_log(s: "Session", res: Dict[str, Any], mu_0: float) -> None:
    """The reference's debug lines, replayed from the recorded history after the solve so the
    hot loop never formats or syncs for them: ``new mu=`` at each phase start
    (gl_ProxGD_primal.py:54) and every 100th iteration ``iter= k, objective= f_hist[k-1],
    sparsity= <of the updated x>`` (:134-136), skipping the iteration where the stop rule broke
    (it does no update, :124-125). SGD/GD's sparsity is recorded at those iterations only."""
    sp, starts, breaks = s.trace()
    f_hist = res["f_hist"]
    k = len(f_hist)
    for p, mu in enumerate((100 * mu_0, 10 * mu_0, mu_0)):
        if starts[p] < 0:
            break
        logger.debug("new mu= {:10E}".format(mu))
        end = starts[p + 1] if p < 2 and starts[p + 1] >= 0 else k
        for it in range(starts[p] + 1, end + 1):
            if it % 100 or it > k or (breaks[p] and it == end):
                continue
            logger.debug("iter= {:5}, objective= {:10E}, sparsity= {:3f}".format(
                it, float(f_hist[it - 1]), float(sp[it - 1]) if it - 1 < len(sp) else float("nan")))


class Session:
    """A solver run split into steps (one step = one recorded iteration).

    ``x`` (device tensor, n x l) holds x0 on entry and is updated in place; A and b must stay
    alive for the session's lifetime. Used by ``bench.py`` to time exactly K iterations.
    """

    def __init__(self, name: str, x: torch.Tensor, A: torch.Tensor, b: torch.Tensor, mu0: float,
                 opts: Dict[str, Any], comm=None):
        method = _lib.METHODS[name]
        if A.dim() != 2 or b.dim() != 2 or x.dim() != 2:
            raise ValueError("A, b and x must be 2-D (group lasso with l columns)")
        m, n = A.shape
        if b.shape[0] != m or x.shape[0] != n or b.shape[1] != x.shape[1]:
            raise ValueError("shape mismatch: A %s, b %s, x %s" % (tuple(A.shape), tuple(b.shape),
                                                                  tuple(x.shape)))
        if not (A.dtype == b.dtype == x.dtype) or A.dtype not in (torch.float32, torch.float64):
            raise ValueError("A, b, x must share dtype float32 or float64")
        for t in (A, b, x):
            if not t.is_cuda or not t.is_contiguous():
                raise ValueError("A, b, x must be contiguous device tensors")
        self.o = make_opts(method, opts)
        if method in (_lib.GLX_SGD, _lib.GLX_GD) and opts.get("continuous_subgradient_flag"):
            self.o.alpha0 = 1.0 / _lambda_max(A, comm)
        self.refs = (A, b, x)
        self.p = GlxProblem(dtype=_lib.GLX_F64 if A.dtype == torch.float64 else _lib.GLX_F32,
                            method=method, m=m, n=n, l=x.shape[1], A=A.data_ptr(), b=b.data_ptr(),
                            x=x.data_ptr(), mu0=float(mu0),
                            comm=comm.handle if comm is not None else None)
        self.device = A.device
        self.ws = workspace(self.p, self.o, self.device)
        self.stream = torch.cuda.current_stream(self.device)
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            check(lib().glx_session_create(ctypes.byref(h), ctypes.byref(self.p), ctypes.byref(self.o),
                                           ctypes.c_void_p(self.ws.data_ptr()), self.ws.numel(),
                                           ctypes.c_void_p(self.stream.cuda_stream)))
        self.h = h
        self.finished = False
        self.steps = 0

    def run(self, steps: int = 0) -> int:
        """Run up to ``steps`` iterations (0 = to completion). Returns iterations run."""
        done = ctypes.c_int64(0)
        fin = ctypes.c_int32(0)
        with torch.cuda.device(self.device):
            check(lib().glx_session_run(self.h, int(steps), ctypes.byref(done), ctypes.byref(fin)))
        self.finished = bool(fin.value)
        self.steps += done.value
        return done.value

    def kernel_time(self, kind: int) -> Tuple[int, float]:
        """(launches timed, total ms) of A@x (0: the dense pass) / A^T r (1) / the split-candidate
        A e gather (2): every k-th launch of that kind with opts profile=k."""
        cnt = ctypes.c_int64(0)
        ms = ctypes.c_double(0)
        check(lib().glx_session_kernel_time(self.h, kind, ctypes.byref(cnt), ctypes.byref(ms)))
        return cnt.value, ms.value

    def counters(self) -> Dict[str, int]:
        """Cumulative executed work: A@x passes, their right-hand sides, A^T r passes, readbacks."""
        out = (ctypes.c_int64 * 4)()
        check(lib().glx_session_counters(self.h, out))
        return {"ax_calls": out[0], "ax_sources": out[1], "atr_calls": out[2], "syncs": out[3]}

    def progress(self) -> Dict[str, int]:
        """Thread-safe progress record (glx_session_progress), for watchdogs: iterations so far,
        phase, what the host waits on (0 nothing, 1 packet, 2 decision record), collectives
        issued."""
        h = getattr(self, "h", None)
        if not h:
            return {"closed": 1}
        out = (ctypes.c_int64 * 4)()
        check(lib().glx_session_progress(h, out))
        return {"k": out[0], "phase": out[1], "waiting_on": out[2], "collectives_issued": out[3]}

    def describe(self) -> str:
        """The kernels this session launches (glx_session_describe): A@X tiles per right-hand
        side count, A^T r panel (+ the fused trial), the split-candidate form, the device-control
        window."""
        buf = ctypes.create_string_buffer(1024)
        check(lib().glx_session_describe(self.h, buf, len(buf)))
        return buf.value.decode()

    def split_trace(self) -> np.ndarray:
        """Per trial batch: ProxGD's flagged rows of e, FProxGD's nnz(e_c) of a gathered batch
        (row form: flagged rows) or -1 for a dense batch (glx_session_split_trace)."""
        n = ctypes.c_int64(0)
        check(lib().glx_session_split_trace(self.h, None, 0, ctypes.byref(n)))
        out = np.zeros(int(n.value), dtype=np.float64)
        if n.value:
            check(lib().glx_session_split_trace(self.h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                                int(n.value), ctypes.byref(n)))
        return out

    def trace(self) -> Tuple[np.ndarray, List[int], List[int]]:
        """(sparsity after each iteration's update, phase start k's, phases ended by the stop rule)
        — see glx_session_trace; valid after finish()."""
        n = ctypes.c_int64(0)
        info = (ctypes.c_int64 * 6)()
        check(lib().glx_session_trace(self.h, None, 0, ctypes.byref(n), info))
        sp = np.full(int(n.value), np.nan)
        if n.value:
            check(lib().glx_session_trace(self.h, sp.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                          int(n.value), ctypes.byref(n), info))
        return sp, [int(v) for v in info[:3]], [int(v) for v in info[3:]]

    def finish(self) -> Dict[str, Any]:
        cap = max(1, 3 * int(self.o.maxit))
        if self.o.max_total_iters > 0:
            cap = min(cap, int(self.o.max_total_iters))
        fh = np.zeros(cap, dtype=np.float64)
        fb = np.zeros(cap, dtype=np.float64)
        res = GlxResult(f_hist=fh.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                        f_hist_best=fb.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), f_cap=cap)
        with torch.cuda.device(self.device):
            check(lib().glx_session_finish(self.h, ctypes.byref(res)))
        n = int(res.n_fhist)
        return {"k": int(res.iters), "fval": np.float64(res.fval), "tt": float(res.tt),
                "f_hist": [np.float64(v) for v in fh[:n]],
                "f_hist_best": [np.float64(v) for v in fb[:n]],
                "ax_calls": int(res.ax_calls), "atr_calls": int(res.atr_calls),
                "syncs": int(res.syncs), "ax_sources": int(res.ax_sources),
                "record_waits": int(res.record_waits),
                "stats": [float(v) for v in res.stats]}

    def close(self):
        if getattr(self, "h", None):
            lib().glx_session_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def solve(name: str, x0, A, b, mu_0, opts: Optional[Dict[str, Any]] = None, comm=None
          ) -> Tuple[Any, int, Dict[str, Any]]:
    """Run ``name`` (e.g. ``"gl_ProxGD_primal"``) on the GPU; reference-compatible return."""
    opts = dict(opts or {})
    if name not in _lib.METHODS:
        raise ValueError("unknown solver %r" % (name,))
    if int(opts.get("shard_model", 0)) > 1:
        raise ValueError("shard_model is bench.py's per-rank timing model (its iterates are not a "
                         "solve); solve() refuses it")
    lib()  # fail loudly before touching data if the library is missing
    device = _device(opts)
    dtype = _dtype_of(A)
    numpy_in = not isinstance(x0, torch.Tensor)
    Ad = _as_device(A, device, dtype)
    bd = _as_device(b, device, dtype)
    xd = _as_device(x0, device, dtype).clone()      # x = np.copy(x0)  (gl_ProxGD_primal.py:49)
    s = Session(name, xd, Ad, bd, float(mu_0), opts, comm=opts.get("comm", comm))
    logger.debug("alpha0= {:10E}".format(s.o.alpha0))
    try:
        s.run(0)
        res = s.finish()
        plan = s.describe()
        if logger.isEnabledFor(logging.DEBUG):
            _replay_log(s, res, float(mu_0))
    finally:
        s.close()
    torch.cuda.synchronize(device)
    x = xd.cpu().numpy() if numpy_in else xd
    out = {"tt": res["tt"], "fval": res["fval"], "f_hist": res["f_hist"],
           "f_hist_best": res["f_hist_best"],
           "glx": {"ax_calls": res["ax_calls"], "atr_calls": res["atr_calls"], "syncs": res["syncs"],
                   "plan": plan}}
    return x, res["k"], out
