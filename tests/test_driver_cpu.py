"""The main.py-parity driver (glx/driver.py) checked on the CPU.

The driver's reporting (main.py:113-130 log line, main.py:94-110 table) is exercised with the
oracle's solvers injected through ``run(solvers=...)``; the product registry itself is GPU-only
(tests/test_gpu_driver.py). The table the driver prints is compared with the report's own
Statistics table (tests/golden/report_table.json, transcribed from doc/report.md:439-447), and
the x* fixture that replaces the CVX columns is checked against the report's CVX-Mosek row.
"""
import io
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

ORDER = ["SGD Primal", "GD Primal", "FGD Primal", "ProxGD Primal", "FProxGD Primal"]
METHOD = {"SGD Primal": "gl_SGD_primal", "GD Primal": "gl_GD_primal", "FGD Primal": "gl_FGD_primal",
          "ProxGD Primal": "gl_ProxGD_primal", "FProxGD Primal": "gl_FProxGD_primal"}


def _report():
    with open(os.path.join(GOLDEN, "report_table.json")) as fh:
        rep = json.load(fh)
    cols = rep["columns"]
    return {k: dict(zip(cols, v)) for k, v in rep["rows"].items()}


def _xstar():
    with np.load(os.path.join(GOLDEN, "default_xstar.npz")) as z:
        return z["x"], float(z["residual"])


def check_against_report(log_dicts, xstar_col=True, fgd_k_rel=0.0):
    """The columns main.py prints, compared as the strings main.py formats.

    FGD's k on this instance is decided by ulp-level summation order (parity
    section); ``fgd_k_rel`` allows the GPU path the same 0.5% the parity suite allows.
    """
    rep = _report()
    assert list(log_dicts) == ORDER
    for mode, d in log_dicts.items():
        want = rep[mode]
        assert list(d) == ["cpu", "iter", "optval", "sparsity", "err-to-exact", "err-to-x*"]
        it = int(d["iter"])
        if mode == "FGD Primal":      # 2034 in this image's reference run (report: 2037, see fixture)
            assert abs(it - 2034) <= fgd_k_rel * 2034, d
        else:
            assert it == int(want["iter"]), (mode, d)
        for key in ("optval", "sparsity", "err-to-exact"):
            assert d[key] == want[key], (mode, key, d[key], want[key])
        if xstar_col:                 # x* ~ CVX-Mosek's point: same leading digit and exponent
            got, ref = float(d["err-to-x*"]), float(want["err-to-cvx-mosek"])
            assert 0.9 < got / ref < 1.1, (mode, got, ref)


def test_gen_data_matches_oracle():
    from glx import driver
    from oracle import numpy_ref
    n, m, l, mu, A, b, u, x0, *_ = driver.gen_data()
    A2, b2, u2, x02, mu2 = numpy_ref.gen_data()
    assert (m, n, l, mu) == (256, 512, 2, mu2)
    for a, c in ((A, A2), (b, b2), (u, u2), (x0, x02)):
        assert np.array_equal(a, c)


def test_xstar_fixture_reproduces_cvx_row():
    from glx import driver
    from oracle import numpy_ref
    xs, res = _xstar()
    n, m, l, mu, A, b, u, x0, errfun, errfun_exact, sparsity = driver.gen_data()
    assert res < 1e-11
    # re-certify: proximal fixed point of the group-lasso objective at mu
    L = float(np.linalg.norm(A, 2)) ** 2
    w = xs - (A.T @ (A @ xs - b)) / L
    nrm = np.linalg.norm(w, axis=1, keepdims=True)
    prox = w * np.maximum(nrm - mu / L, 0) / np.where(nrm > 0, nrm, 1)
    assert np.linalg.norm(xs - prox) * L < 1e-10
    rep = _report()["CVX-Mosek"]
    assert "%6.4f" % sparsity(xs) == rep["sparsity"]
    assert "%3.2E" % errfun_exact(xs) == rep["err-to-exact"]
    assert "%6.5E" % driver.obj_func(A, b, mu, xs) == rep["optval"]
    # every solver in the report stops at or above the minimum
    for name in ("gl_ProxGD_primal", "gl_FProxGD_primal"):
        x, _, out = numpy_ref.SOLVERS[name](x0.copy(), A, b, mu, {})
        assert out["fval"] >= driver.obj_func(A, b, mu, xs) - 1e-12


def test_driver_table_with_oracle_solvers_matches_report(tmp_path):
    from glx import driver
    from oracle import numpy_ref
    solvers = {mode: numpy_ref.SOLVERS[METHOD[mode]] for mode in ORDER}
    buf = io.StringIO()
    res = driver.run(solvers, xstar=_xstar()[0], dest_dir=str(tmp_path), stream=buf)
    check_against_report(res["log_dicts"])
    text = buf.getvalue().splitlines()
    assert text[0] == "# Statistics"
    assert text[1].split("|")[1].strip() == "solver" and len(text) == 3 + len(ORDER)
    assert all(line.startswith("|") and line.endswith("|") for line in text[1:])
    with np.load(tmp_path / "f_hist.npz") as z:
        assert set(z.files) == {"f_star"} | {m.replace(" ", "_") for m in ORDER}
        assert len(z["ProxGD_Primal"]) == 1768


def test_log_line_format(caplog):
    from glx import driver
    _, _, _, _, _, _, u, x0, errfun, errfun_exact, sparsity = driver.gen_data()
    fake = lambda x0, A, b, mu, opts: (x0, None, {"tt": 1.234, "fval": 0.5})
    with caplog.at_level("INFO", logger=driver.LOGGER):
        _, _, _, d = driver.solve_routine("ProxGD Primal", fake, x0, None, None, 1e-2, {},
                                          errfun, errfun_exact, sparsity)
    assert d["iter"] == "   -1" and d["cpu"] == " 1.23" and d["err-to-x*"] == "n/a"
    assert caplog.records[-1].getMessage().startswith("[ProxGD Primal]: cpu:  1.23, iter:    -1, optval: 5.00000E-01")


def test_cli_rejects_unknown_solver():
    from glx import driver
    with pytest.raises(SystemExit):
        driver.main(["--solvers", "ADMM Dual", "--log", ""])
