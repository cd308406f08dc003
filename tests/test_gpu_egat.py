"""Round 6: the split-candidate ProxGD trial with A e fused into the dense pass (launch_ax_egat,
kernels_axdma.hip; gl_ProxGD_primal.py:89-92 g(z) and :112 the objective of the candidate, from
A p = A p_thr + A e).

The fused pass streams A p on MFMA (the objective and the Armijo test directly) and A e on VALU
from the same LDS chunks; the next gradient residual is (A p - b) - A e instead of the gather
form's direct A p_thr - b (GLX_AE_FUSED=0: the transposed copy of A and k_at_gather_bm), so the two
forms agree to rounding (k identical, f_hist within 1e-11, x within 1e-9 of max|x|). Against the
oracle: the north-star bar (k identical, f_hist within 1e-8, x within 1e-6 of max|x|).

Round 6, the per-trial choice (GLX_AE_HYB_ROWS, default 2000 flagged rows; one GPU, host control,
the NS tile): the gather while few rows are flagged, the fused form from the threshold on. Forced
early here (100 rows) so both forms and the switch run within a short solve.
"""
import warnings

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


def _run(monkeypatch, fused, A, b, x0, mu, opts, hyb="0"):
    from gl_ProxGD_primal import gl_ProxGD_primal
    monkeypatch.setenv("GLX_AE_FUSED", "1" if fused else "0")
    monkeypatch.setenv("GLX_AE_HYB_ROWS", hyb)   # "0": the gather throughout (not per trial)
    x, k, out = gl_ProxGD_primal(torch.from_numpy(x0).cuda(), A, b, mu, dict(opts))
    torch.cuda.synchronize()
    return x.cpu().numpy(), k, np.asarray([float(v) for v in out["f_hist"]]), out["glx"]["plan"]


@pytest.mark.parametrize("l,maxit", [(32, 40), (16, 10)])
def test_fused_ae_matches_gather_and_oracle(monkeypatch, l, maxit):
    from oracle import numpy_ref
    m, n = 8192, 16384
    A, b, u, x0, mu = numpy_ref.gen_data(m, n, l, 97006855)
    opts = {"alpha0": numpy_ref.step_size_for(m, n), "maxit": maxit}
    At, bt = torch.from_numpy(A).cuda(), torch.from_numpy(b).cuda()
    xf, kf, ff, pf = _run(monkeypatch, True, At, bt, x0, mu, opts)
    xg, kg, fg, pg = _run(monkeypatch, False, At, bt, x0, mu, opts)
    assert "A e fused into the dense pass" in pf, pf
    assert "gather k_at_gather_bm" in pg, pg
    assert kf == kg == 3 * maxit
    assert np.max(np.abs(xf - xg)) <= 1e-9 * np.max(np.abs(xg))
    assert np.max(np.abs(ff - fg) / np.abs(fg)) < 1e-11
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        xr, kr, outr = numpy_ref.gl_ProxGD_primal(x0, A, b, mu, dict(opts))
    fr = np.asarray([float(v) for v in outr["f_hist"]])
    assert kf == kr
    assert np.max(np.abs(ff - fr) / np.abs(fr)) < 1e-8
    assert np.max(np.abs(xf - xr)) <= 1e-6 * np.max(np.abs(xr))


def test_fused_ae_rejections(monkeypatch):
    """alpha0 = 2.5 / L: rejected first trials (the retrial's k_prox_pgd writes p and its bitmaps,
    the fused pass reads them): the gather form's iterates to rounding, 20 per phase."""
    from oracle import numpy_ref
    m, n, l = 8192, 16384, 32
    A, b, u, x0, mu = numpy_ref.gen_data(m, n, l, 5)
    opts = {"alpha0": 2.5 * numpy_ref.step_size_for(m, n), "maxit": 20}
    At, bt = torch.from_numpy(A).cuda(), torch.from_numpy(b).cuda()
    xf, kf, ff, _ = _run(monkeypatch, True, At, bt, x0, mu, opts)
    xg, kg, fg, _ = _run(monkeypatch, False, At, bt, x0, mu, opts)
    assert kf == kg
    assert np.max(np.abs(xf - xg)) <= 1e-9 * np.max(np.abs(xg))
    assert np.max(np.abs(ff - fg) / np.abs(fg)) < 1e-11


def test_hybrid_form_switches_and_matches_oracle(monkeypatch):
    from oracle import numpy_ref
    m, n, l, maxit = 8192, 16384, 32, 40
    A, b, u, x0, mu = numpy_ref.gen_data(m, n, l, 97006855)
    opts = {"alpha0": numpy_ref.step_size_for(m, n), "maxit": maxit}
    At, bt = torch.from_numpy(A).cuda(), torch.from_numpy(b).cuda()
    xh, kh, fh, ph = _run(monkeypatch, False, At, bt, x0, mu, opts, hyb="100")
    xg, kg, fg, _ = _run(monkeypatch, False, At, bt, x0, mu, opts, hyb="0")
    assert "from 100 flagged rows" in ph, ph
    assert kh == kg == 3 * maxit
    assert np.max(np.abs(xh - xg)) <= 1e-9 * np.max(np.abs(xg))
    assert np.max(np.abs(fh - fg) / np.abs(fg)) < 1e-11
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        xr, kr, outr = numpy_ref.gl_ProxGD_primal(x0, A, b, mu, dict(opts))
    fr = np.asarray([float(v) for v in outr["f_hist"]])
    assert kh == kr
    assert np.max(np.abs(fh - fr) / np.abs(fr)) < 1e-8
    assert np.max(np.abs(xh - xr)) <= 1e-6 * np.max(np.abs(xr))
