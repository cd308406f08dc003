"""Split-candidate ProxGD (A p = A p_thr + A e, the bitmap gather k_at_gather_bm) at ragged n,
with a workspace that starts as all-ones bytes.

The bitmap gather reads every u64 word of each column bitmap up to ceil64(n) rows; the trial
kernels write only the row groups they visit (the 16-row groups below ceil16(n), the 64 / 32-row
A^T R panels). Words of rows >= n that no trial writes must read as zero, or the gather reads
At and E beyond n and corrupts A e, the Armijo test and the recorded objective. The session
clears zf at creation and the gather masks rows >= n itself; these tests fill the workspace with
0xFF bytes first (the worst stale content torch.empty could hand back) and compare the whole
trajectory with the oracle (gl_ProxGD_primal.py:73-132) at the fp64 bar.
  - n = 1000 (n % 64 = 40): groups [1008, 1024) are never visited by the 16-row trials;
  - n = 8224 (n % 64 = 32): the 16-row trial kernels never write the groups of rows
    [8224, 8256) — the upper half of the last u64 of every column bitmap.
"""
import warnings

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


@pytest.fixture
def dirty_workspace(monkeypatch):
    import glx.solver as gs
    orig = gs.workspace

    def filled(problem, o, device):
        ws = orig(problem, o, device)
        ws.fill_(0xFF)
        return ws
    monkeypatch.setattr(gs, "workspace", filled)


def _rel(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return float(np.max(np.abs(a - b) / np.abs(b)))


@pytest.mark.parametrize("m,n,maxit", [(512, 1000, 2500), (1024, 8224, 40)])
def test_ragged_split_candidate_vs_oracle(dirty_workspace, m, n, maxit):
    from oracle import numpy_ref
    from gl_ProxGD_primal import gl_ProxGD_primal
    l = 32
    A, b, u, x0, mu = numpy_ref.gen_data(m, n, l, 4242)
    opts = {"alpha0": numpy_ref.step_size_for(m, n), "maxit": maxit, "split_cand": 1}
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        xr, kr, outr = numpy_ref.gl_ProxGD_primal(x0, A, b, mu, dict(opts))
    x, k, out = gl_ProxGD_primal(x0, A, b, mu, dict(opts))
    plan = out["glx"]["plan"]
    assert "k_at_gather_bm" in plan, plan
    assert k == kr, (k, kr)
    assert _rel(out["fval"], outr["fval"]) < 1e-8
    assert _rel([float(v) for v in out["f_hist"]], [float(v) for v in outr["f_hist"]]) < 1e-8
    assert np.max(np.abs(x - xr)) <= 1e-6 * np.max(np.abs(xr))
