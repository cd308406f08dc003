"""The line-search trials fused into A^T r (k_atr_prox for ProxGD, k_atr_fista for FProxGD) and
their speculative use.

At (m, n, l) = (256, 16384, 32) fp64 the planner gives A^T r one K split, so the solver runs
the first line-search trial of every iteration inside the gradient kernel's epilogue and, after
an accepted first trial, queues the next iteration's fused kernel before the host has read
the trial's scalars. Per element the fused epilogue does exactly k_prox_pgd's arithmetic on the
same gradient, so the iterate must be bit-identical to the unfused path (GLX_FUSED_TRIAL=0);
only the grid-sum order of the trial's scalars differs (ulp-level f_hist differences). Against
the NumPy oracle the bar is the north-star 1e-8 on the objective.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

SHAPE = (256, 16384, 32)


def _instance():
    from oracle import numpy_ref
    m, n, l = SHAPE
    A, b, u, x0, mu = numpy_ref.gen_data(m, n, l, 2024)
    return A, b, x0, mu, numpy_ref.step_size_for(m, n)


METHODS = ["gl_ProxGD_primal", "gl_FProxGD_primal"]


def _run(monkeypatch, fused, spec, opts, method="gl_ProxGD_primal"):
    import glx
    monkeypatch.setenv("GLX_FUSED_TRIAL", "1" if fused else "0")
    monkeypatch.setenv("GLX_SPEC_GRAD", "1" if spec else "0")
    A, b, x0, mu, _ = _instance()
    At, bt, xt = (torch.from_numpy(a).cuda() for a in (A, b, x0))
    s = glx.Session(method, xt, At, bt, mu, opts)
    s.run(0)
    res = s.finish()
    s.close()
    torch.cuda.synchronize()
    return xt.cpu().numpy(), res


def test_plan_fuses_at_this_shape():
    from glx import _lib
    d = _lib.plan_describe(_lib.GLX_F64, *SHAPE)
    assert "atr=k_atr_mfma<WL0" in d and d.rstrip().endswith("S=1"), d


@pytest.mark.parametrize("method", METHODS)
@pytest.mark.parametrize("spec", [False, True])
def test_fused_trial_bit_identical_iterate(monkeypatch, spec, method):
    _, _, _, _, alpha0 = _instance()
    opts = {"alpha0": alpha0, "maxit": 40}
    x_f, r_f = _run(monkeypatch, True, spec, opts, method)
    x_u, r_u = _run(monkeypatch, False, False, opts, method)
    assert r_f["k"] == r_u["k"]
    assert np.array_equal(x_f, x_u)
    np.testing.assert_allclose(np.asarray(r_f["f_hist"]), np.asarray(r_u["f_hist"]), rtol=1e-13)
    if spec:   # every accepted first trial queued the next fused kernel
        assert r_f["atr_calls"] >= r_u["atr_calls"]


@pytest.mark.parametrize("method", METHODS)
def test_fused_trial_matches_oracle(monkeypatch, method):
    from oracle import numpy_ref
    A, b, x0, mu, alpha0 = _instance()
    opts = {"alpha0": alpha0, "maxit": 25}
    x_g, r_g = _run(monkeypatch, True, True, opts, method)
    x_r, k_r, out_r = numpy_ref.SOLVERS[method](x0.copy(), A, b, mu, dict(opts))
    assert r_g["k"] == k_r
    f_g = np.asarray(r_g["f_hist"], dtype=float)
    f_r = np.asarray(out_r["f_hist"], dtype=float)
    assert np.max(np.abs(f_g - f_r) / np.abs(f_r)) < 1e-8
    assert abs(float(r_g["fval"]) - float(out_r["fval"])) <= 1e-8 * abs(float(out_r["fval"]))


@pytest.mark.parametrize("method", METHODS)
def test_fused_trial_fixed_step(monkeypatch, method):
    _, _, _, _, alpha0 = _instance()
    opts = {"alpha0": alpha0, "maxit": 20, "step_type": "fixed"}
    x_f, r_f = _run(monkeypatch, True, True, opts, method)
    x_u, r_u = _run(monkeypatch, False, False, opts, method)
    assert r_f["k"] == r_u["k"]
    assert np.array_equal(x_f, x_u)


# K-split fused kernels (round 3): with S > 1 only the panel owners (the last arriver of each
# panel's S blocks) and the publisher join the trial's grid reduction, so S is no longer bounded
# by the 1024-slot partials row (C2 = 128 panels could not take 8 splits before). G is summed
# over the S slabs in slab order in both paths, so the iterate is bit-identical to the unfused
# kernels at the same S; the scalars' panel order is fixed whatever the arrival order.
SPLIT_SHAPE = (1024, 8192, 16)


@pytest.mark.parametrize("method", METHODS)
@pytest.mark.parametrize("S", [2, 4, 8])
@pytest.mark.parametrize("dc", [0, 8])
def test_fused_trial_k_splits(monkeypatch, method, S, dc):
    import glx
    from oracle import numpy_ref
    m, n, l = SPLIT_SHAPE
    A, b, u, x0, mu = numpy_ref.gen_data(m, n, l, 77)
    opts = {"alpha0": numpy_ref.step_size_for(m, n), "maxit": 30, "dc_window": dc}
    monkeypatch.setenv("GLX_ATR_S", str(S))
    from glx import _lib
    assert _lib.plan_describe(_lib.GLX_F64, m, n, l).rstrip().endswith("S=%d" % S)

    def run(fused):
        monkeypatch.setenv("GLX_FUSED_TRIAL", "1" if fused else "0")
        At, bt, xt = (torch.from_numpy(a).cuda() for a in (A, b, x0))
        s = glx.Session(method, xt, At, bt, mu, opts)
        s.run(0)
        res = s.finish()
        s.close()
        torch.cuda.synchronize()
        return xt.cpu().numpy(), res

    x_f, r_f = run(True)
    x_u, r_u = run(False)
    assert r_f["k"] == r_u["k"]
    assert np.array_equal(x_f, x_u)
    np.testing.assert_allclose(np.asarray(r_f["f_hist"]), np.asarray(r_u["f_hist"]), rtol=1e-13)
    x_2, r_2 = run(True)   # run to run: bit-identical scalars and iterate
    assert np.array_equal(x_f, x_2) and list(r_f["f_hist"]) == list(r_2["f_hist"])
    x_r, k_r, out_r = numpy_ref.SOLVERS[method](x0.copy(), A, b, mu, {k: v for k, v in opts.items() if k != "dc_window"})
    assert r_f["k"] == k_r
    f_g, f_r = np.asarray(r_f["f_hist"], dtype=float), np.asarray(out_r["f_hist"], dtype=float)
    assert np.max(np.abs(f_g - f_r) / np.abs(f_r)) < 1e-8


# Round 4: the eight-wave panel (A^T R code 1028: WL 2, two waves per SIMD) in the fused
# kernels, with one and two K splits: the iterate stays bit-identical to the unfused path on the
# same tile, and within the north-star bar of the oracle.
@pytest.mark.parametrize("method", METHODS)
@pytest.mark.parametrize("S", [1, 2])
def test_fused_trial_eight_wave_panel(monkeypatch, method, S):
    from oracle import numpy_ref
    from glx import _lib
    monkeypatch.setenv("GLX_ATR_VARIANT", "1028")
    monkeypatch.setenv("GLX_ATR_S", str(S))
    d = _lib.plan_describe(_lib.GLX_F64, *SHAPE)
    assert "WL2" in d and d.rstrip().endswith("S=%d" % S), d
    A, b, x0, mu, alpha0 = _instance()
    opts = {"alpha0": alpha0, "maxit": 25}
    x_f, r_f = _run(monkeypatch, True, True, opts, method)
    x_u, r_u = _run(monkeypatch, False, False, opts, method)
    assert r_f["k"] == r_u["k"]
    assert np.array_equal(x_f, x_u)
    np.testing.assert_allclose(np.asarray(r_f["f_hist"]), np.asarray(r_u["f_hist"]), rtol=1e-13)
    x_r, k_r, out_r = numpy_ref.SOLVERS[method](x0.copy(), A, b, mu, dict(opts))
    assert r_f["k"] == k_r
    f_g, f_r = np.asarray(r_f["f_hist"], dtype=float), np.asarray(out_r["f_hist"], dtype=float)
    assert np.max(np.abs(f_g - f_r) / np.abs(f_r)) < 1e-8


# Round 5: the 32-column A^T R panel (WL 3: four waves, f64, one K split; its eight-wave form WL 4
# was pruned in round 6) in the fused kernels: the iterate is bit-identical to the unfused path on
# the same tile and within the north-star bar of the oracle.
@pytest.mark.parametrize("code,wl", [("38", "WL3"), ("1038", "WL3")])
@pytest.mark.parametrize("method", METHODS)
def test_fused_trial_narrow_panel(monkeypatch, method, code, wl):
    from oracle import numpy_ref
    from glx import _lib
    monkeypatch.setenv("GLX_ATR_VARIANT", code)
    monkeypatch.setenv("GLX_ATR_S", "1")
    d = _lib.plan_describe(_lib.GLX_F64, *SHAPE)
    assert wl in d and "S=1" in d, d
    A, b, x0, mu, alpha0 = _instance()
    opts = {"alpha0": alpha0, "maxit": 25}
    x_f, r_f = _run(monkeypatch, True, True, opts, method)
    x_u, r_u = _run(monkeypatch, False, False, opts, method)
    assert r_f["k"] == r_u["k"]
    assert np.array_equal(x_f, x_u)
    np.testing.assert_allclose(np.asarray(r_f["f_hist"]), np.asarray(r_u["f_hist"]), rtol=1e-13)
    x_r, k_r, out_r = numpy_ref.SOLVERS[method](x0.copy(), A, b, mu, dict(opts))
    assert r_f["k"] == k_r
    f_g, f_r = np.asarray(r_f["f_hist"], dtype=float), np.asarray(out_r["f_hist"], dtype=float)
    assert np.max(np.abs(f_g - f_r) / np.abs(f_r)) < 1e-8


def test_session_plan_takes_narrow_panel_at_c2():
    """C2's shape (4096, 8192, 16): 128 64-column panels, so the session plans 256 32-column
    panels without K splits for the fused trial (GLX_ATR_NARROW=0: the 2-split 64-column form)."""
    import glx
    m, n, l = 4096, 8192, 16
    A = torch.zeros(m, n, dtype=torch.float64, device="cuda")
    b = torch.zeros(m, l, dtype=torch.float64, device="cuda")
    x = torch.zeros(n, l, dtype=torch.float64, device="cuda")
    s = glx.Session("gl_ProxGD_primal", x, A, b, 1e-2, {"alpha0": 1e-5})
    d = s.describe()
    s.close()
    assert "atr=k_atr_mfma<WL3,PF8" in d and "S=1" in d and "+trial (k_atr_prox)" in d, d
