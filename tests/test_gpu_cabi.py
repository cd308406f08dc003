"""The ctypes stub of INTEGRATION.md §2, run as written against the raw C ABI (glx_solve).

The stub is read out of INTEGRATION.md at test time, so the document cannot drift from the ABI.
It must reproduce the reference's golden ProxGD run on the default instance.
"""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from conftest import ROOT, golden_case, golden_inputs

pytestmark = pytest.mark.gpu


def _stub_namespace():
    md = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    i = md.index("```python\nimport ctypes, numpy as np, torch")
    j = md.index("```", i + 10)
    src = md[i + len("```python\n"):j]
    ns = {}
    cwd = os.getcwd()
    os.chdir(ROOT)   # the stub loads the library by its repo-relative path
    try:
        exec(compile(src, "INTEGRATION.md", "exec"), ns)
    finally:
        os.chdir(cwd)
    return ns


def test_integration_stub_matches_golden():
    ns = _stub_namespace()
    meta, gold = golden_case("default_gl_ProxGD_primal")
    A, b, u, x0, mu = golden_inputs(meta)
    x, k, out = ns["gl_ProxGD_primal"](x0, A, b, mu, {})
    assert k == int(gold["k"])
    assert abs(out["fval"] - float(gold["fval"])) <= 1e-8 * abs(float(gold["fval"]))
    np.testing.assert_allclose(np.asarray(out["f_hist"]), gold["f_hist"], rtol=1e-8)
    assert x.shape == x0.shape
