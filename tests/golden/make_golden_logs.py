"""Record the reference solvers' 'opt' logger lines (DEBUG) as a fixture: tests/golden/logs.json.

Run in the build container only (imports the reference from /root/reference/code, like
make_golden.py; no reference source is stored — only the emitted text lines):

    python tests/golden/make_golden_logs.py

The lines are `alpha0=`, `new mu=` per phase (gl_ProxGD_primal.py:45,54) and the every-100th-
iteration `iter= ..., objective= ..., sparsity= ...` line (:134-136), for the default instance of
every solver and one other seed. tests/test_oracle.py checks the oracle's restated lines against
them; tests/test_gpu_logs.py checks the HIP solvers' replayed lines.
"""
from __future__ import annotations

import json
import logging
import os
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

from make_golden import REF_SOLVERS  # noqa: E402  (imports the reference solvers)
from oracle.numpy_ref import gen_data  # noqa: E402

CASES = [("default_" + s, s, 97006855) for s in REF_SOLVERS] + \
        [("seed114514_gl_ProxGD_primal", "gl_ProxGD_primal", 114514)]


class _Grab(logging.Handler):
    def __init__(self):
        super().__init__(logging.DEBUG)
        self.lines = []

    def emit(self, rec):
        self.lines.append(rec.getMessage())


def main():
    log = logging.getLogger("opt")
    log.setLevel(logging.DEBUG)
    out = {}
    for name, solver, seed in CASES:
        h = _Grab()
        log.addHandler(h)
        A, b, u, x0, mu = gen_data(256, 512, 2, seed)
        REF_SOLVERS[solver](x0, A, b, mu, {})
        log.removeHandler(h)
        out[name] = {"solver": solver, "seed": seed, "m": 256, "n": 512, "l": 2, "lines": h.lines}
        print(name, len(h.lines))
    with open(os.path.join(HERE, "logs.json"), "w") as fh:
        json.dump(out, fh, indent=0)


if __name__ == "__main__":
    main()
