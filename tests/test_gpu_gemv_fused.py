"""The l = 1 descent pass in one sweep of A (kernels_gemv.hip, SGD / GD, config C4).

k_gemv_pair_fused keeps whole rows of A in registers: it reduces their dot products with x and
thr(x) over the workgroup and adds row * (A thr(x) - b)_i into a per-workgroup slab of the
gradient, so A is read once per iteration instead of twice. Its sums run in a different order
than the two-pass path (A @ [x | thr(x)], then A^T r; GLX_GEMV_FUSED=0), so the two agree to
rounding, not bitwise. Checks: fused vs two-pass and vs the NumPy oracle (k identical, f_hist
within 1e-10 / the north-star 1e-8), run-to-run bit reproducibility, one pass over A per
iteration, and the shapes the kernel treats specially (ragged rows per workgroup, n not a
multiple of the 1024-column thread stride, few rows, fp32).
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


def _run(monkeypatch, fused, method, A, b, x0, mu, opts):
    import glx
    monkeypatch.setenv("GLX_GEMV_FUSED", "1" if fused else "0")
    At, bt, xt = (torch.from_numpy(a).cuda() for a in (A, b, x0))
    s = glx.Session(method, xt, At, bt, mu, opts)
    s.run(0)
    res = s.finish()
    s.close()
    torch.cuda.synchronize()
    return xt.cpu().numpy(), res


def _instance(m, n, dtype=np.float64, seed=5):
    from oracle import numpy_ref
    A, b, u, x0, mu = numpy_ref.gen_data(m, n, 1, seed)
    return A.astype(dtype), b.astype(dtype), x0.astype(dtype), mu, numpy_ref.step_size_for(m, n)


SHAPES = [(4096, 2048), (3001, 1030), (65, 8192), (7, 512), (1031, 256), (2048, 8190)]


@pytest.mark.parametrize("method", ["gl_SGD_primal", "gl_GD_primal"])
@pytest.mark.parametrize("shape", SHAPES)
def test_fused_matches_two_pass_and_oracle(monkeypatch, method, shape):
    from oracle import numpy_ref
    A, b, x0, mu, alpha0 = _instance(*shape)
    opts = {"alpha0": alpha0, "maxit": 12}
    x_f, r_f = _run(monkeypatch, True, method, A, b, x0, mu, opts)
    x_u, r_u = _run(monkeypatch, False, method, A, b, x0, mu, opts)
    assert r_f["k"] == r_u["k"]
    f_f, f_u = np.asarray(r_f["f_hist"]), np.asarray(r_u["f_hist"])
    assert np.max(np.abs(f_f - f_u) / np.abs(f_u)) < 1e-10
    np.testing.assert_allclose(x_f, x_u, rtol=1e-9, atol=1e-12 * np.abs(x_u).max())
    # one pass over A per iteration (plus the prologue); the two-pass path needs two
    assert r_f["atr_calls"] == 0 and r_f["ax_calls"] == r_f["k"] + 2   # + prologue, + finish()
    x_r, k_r, out_r = numpy_ref.SOLVERS[method](x0.copy(), A, b, mu, dict(opts))
    assert r_f["k"] == k_r
    f_r = np.asarray(out_r["f_hist"], dtype=float)
    assert np.max(np.abs(f_f - f_r) / np.abs(f_r)) < 1e-8


def test_fused_deterministic(monkeypatch):
    A, b, x0, mu, alpha0 = _instance(8192, 4096)
    opts = {"alpha0": alpha0, "maxit": 8}
    x1, r1 = _run(monkeypatch, True, "gl_SGD_primal", A, b, x0, mu, opts)
    x2, r2 = _run(monkeypatch, True, "gl_SGD_primal", A, b, x0, mu, opts)
    assert np.array_equal(x1, x2)
    assert np.array_equal(np.asarray(r1["f_hist"]), np.asarray(r2["f_hist"]))


def test_fused_fp32(monkeypatch):
    A, b, x0, mu, alpha0 = _instance(4096, 4096, np.float32)
    opts = {"alpha0": alpha0, "maxit": 8}
    x_f, r_f = _run(monkeypatch, True, "gl_SGD_primal", A, b, x0, mu, opts)
    x_u, r_u = _run(monkeypatch, False, "gl_SGD_primal", A, b, x0, mu, opts)
    assert r_f["k"] == r_u["k"]
    f_f, f_u = np.asarray(r_f["f_hist"]), np.asarray(r_u["f_hist"])
    assert np.max(np.abs(f_f - f_u) / np.abs(f_u)) < 1e-5


def test_fused_not_used_for_wide_n(monkeypatch):
    # n > 8192 (fp64) exceeds the row-in-registers budget: the two-pass path runs
    A, b, x0, mu, alpha0 = _instance(64, 16384)
    opts = {"alpha0": alpha0, "maxit": 3}
    _, r = _run(monkeypatch, True, "gl_SGD_primal", A, b, x0, mu, opts)
    assert r["atr_calls"] > 0
