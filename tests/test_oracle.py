"""The CPU oracle (oracle/numpy_ref.py) against the reference's own outputs.

The fixtures were produced by running the reference solvers (tests/golden/make_golden.py);
the oracle must reproduce them bit-for-bit on this NumPy build (≤1e-13 relative is
accepted to tolerate a different BLAS on another host).
"""
import os
import warnings

import numpy as np
import pytest

from conftest import golden_case, golden_index, golden_inputs
from oracle import numpy_ref

CASES = sorted(golden_index())
# keep the CPU suite to a few seconds: the long default-instance runs are sampled
FAST = [c for c in CASES if not c.startswith(("c1_", "default_gl_GD", "default_gl_SGD",
                                              "seed114514_gl_SGD", "steps_dim"))]


def _close(a, b, rtol):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    both_nan = np.isnan(a) & np.isnan(b)
    same_inf = np.isinf(a) & np.isinf(b) & (np.sign(a) == np.sign(b))
    ok = both_nan | same_inf | (np.abs(a - b) <= rtol * np.maximum(np.abs(b), 1e-300))
    return bool(np.all(ok))


@pytest.mark.parametrize("name", FAST)
def test_oracle_matches_reference(name):
    meta, gold = golden_case(name)
    A, b, u, x0, mu = golden_inputs(meta)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        x, k, out = numpy_ref.SOLVERS[meta["solver"]](x0, A, b, mu, dict(meta["opts"]))
    assert k == int(gold["k"])
    assert len(out["f_hist"]) == k
    rtol = 1e-13 if meta["dtype"] == "f64" else 1e-6
    assert _close(out["f_hist"], gold["f_hist"], rtol)
    assert _close(out["f_hist_best"], gold["f_hist_best"], rtol)
    assert _close(out["fval"], gold["fval"], rtol)
    assert _close(x, gold["x"], max(rtol, 1e-12) if meta["dtype"] == "f64" else 1e-4) or \
        np.allclose(x, gold["x"], rtol=1e-10, atol=1e-12)


def test_gen_data_default_instance_matches_report_shape():
    A, b, u, x0, mu = numpy_ref.gen_data()
    assert A.shape == (256, 512) and b.shape == (256, 2) and x0.shape == (512, 2)
    assert np.count_nonzero(np.linalg.norm(u, axis=1)) == 51     # round(0.1 n)
    assert mu == 1e-2


def test_known_answers_from_report():
    """doc/report.md:446-447 — ProxGD 1768 its, FProxGD 1721 its, optval 6.10377E-01."""
    idx = golden_index()
    assert idx["default_gl_ProxGD_primal"]["k"] == 1768
    assert idx["default_gl_FProxGD_primal"]["k"] == 1721
    assert idx["default_gl_SGD_primal"]["k"] == 6300
    assert idx["default_gl_GD_primal"]["k"] == 7500
    assert "%6.5E" % idx["default_gl_ProxGD_primal"]["fval"] == "6.10377E-01"
    assert "%6.5E" % idx["default_gl_FProxGD_primal"]["fval"] == "6.10377E-01"


def test_unknown_step_type_raises():
    A, b, u, x0, mu = numpy_ref.gen_data(16, 32, 2, 1)
    with pytest.raises(ValueError):
        numpy_ref.gl_ProxGD_primal(x0, A, b, mu, {"step_type": "bogus"})


def test_oracle_log_lines_match_reference():
    """The oracle's restated 'opt' debug lines (alpha0=, new mu= per phase, every 100th
    iteration) equal the reference's own, recorded in tests/golden/logs.json."""
    import json
    import logging
    from conftest import GOLDEN
    from oracle import numpy_ref
    logs = json.load(open(os.path.join(GOLDEN, "logs.json")))
    lg = logging.getLogger("oracle.opt")
    for name, case in logs.items():
        lines = []
        h = logging.Handler(logging.DEBUG)
        h.emit = lambda rec: lines.append(rec.getMessage())
        lg.addHandler(h)
        old = lg.level
        lg.setLevel(logging.DEBUG)
        try:
            A, b, u, x0, mu = numpy_ref.gen_data(case["m"], case["n"], case["l"], case["seed"])
            with np.errstate(all="ignore"):
                numpy_ref.SOLVERS[case["solver"]](x0, A, b, mu, {})
        finally:
            lg.removeHandler(h)
            lg.setLevel(old)
        assert lines == case["lines"], name


def test_ns_golden_fixtures_consistent():
    """The north-star whole-solve fixtures (tests/golden/make_golden_ns.py): f_hist has k
    entries, f_hist_best is its running minimum, and the stored b is the instance's."""
    import hashlib
    import json
    gdir = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    b = np.load(os.path.join(gdir, "ns_instance_b.npz"))["b"]
    for m in ("gl_ProxGD_primal", "gl_FProxGD_primal"):
        meta = json.load(open(os.path.join(gdir, "ns_%s.json" % m)))
        d = np.load(os.path.join(gdir, "ns_%s.npz" % m))
        assert hashlib.sha256(b.tobytes()).hexdigest() == meta["sha256"]["b"]
        assert int(d["k"]) == meta["k"] == len(d["f_hist"]) == len(d["f_hist_best"])
        assert np.array_equal(d["f_hist_best"], np.minimum.accumulate(d["f_hist"]))
        assert float(d["fval"]) == meta["fval"]
        assert d["x"].shape == (meta["n"], meta["l"])
