"""Shared pytest configuration.

Markers:
  gpu — needs a real MI355X (run with ``-m gpu`` on the GPU box); everything else runs on CPU.
"""
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "convex-optimization_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: test needs an MI355X GPU (HIP path)")


def golden_index():
    with open(os.path.join(GOLDEN, "index.json")) as fh:
        return json.load(fh)


def golden_case(name):
    """Return (meta, arrays) for a golden fixture."""
    meta = golden_index()[name]
    with np.load(os.path.join(GOLDEN, name + ".npz")) as z:
        arrs = {k: z[k] for k in z.files}
    return meta, arrs


def golden_inputs(meta):
    """Rebuild the instance of a fixture with the repo's generator and pin it by hash."""
    import hashlib
    from oracle.numpy_ref import gen_data
    A, b, u, x0, mu = gen_data(meta["m"], meta["n"], meta["l"], meta["seed"])
    if meta["dtype"] == "f32":
        A, b, u, x0 = (a.astype(np.float32) for a in (A, b, u, x0))
    for key, arr in (("A", A), ("b", b), ("x0", x0), ("u", u)):
        h = hashlib.sha256(np.ascontiguousarray(arr).tobytes()).hexdigest()
        assert h == meta["sha256"][key], "generator drifted for %s" % key
    return A, b, u, x0, mu


@pytest.fixture(scope="session")
def gindex():
    return golden_index()
