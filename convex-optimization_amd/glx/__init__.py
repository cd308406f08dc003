"""glx — MI355X-native group-lasso first-order solvers.

Public surface:
  * ``solve(name, x0, A, b, mu_0, opts)`` — the reference's ``gl_<method>`` contract
    (also re-exported as the drop-in modules ``gl_ProxGD_primal`` etc. next to this package);
  * ``Session`` — the same solver split into steps (benchmarks);
  * ``kernels`` — single HIP kernels (residual, gradient, prox);
  * ``dist`` — row sharding + RCCL communicator.
"""
from ._lib import LIB_PATH, GlxError, lib  # noqa: F401
from .solver import Session, solve  # noqa: F401

__all__ = ["solve", "Session", "lib", "LIB_PATH", "GlxError"]
