"""Drop-in replacement for the reference's ``code/gl_SGD_primal.py`` (def at line 9).

Same module name, function name, signature and return contract — main.py (or any
caller) imports it unchanged with this directory on sys.path. The computation runs on
the GPU through libglx (glx/solver.py); there is no CPU fallback.
"""
from glx.solver import solve as _solve


def gl_SGD_primal(x0, A, b, mu_0, opts: dict):
    return _solve("gl_SGD_primal", x0, A, b, mu_0, opts)
