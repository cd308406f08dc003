"""Kernel-level numerics of the HIP path against an fp64 reference of the same op.

A @ X - B, A^T R and the group prox, for every code path the planner can pick
(MFMA direct loads, MFMA quad loads + bpermute, MFMA with X staged in LDS, MFMA with A and X
staged by LDS-DMA, VALU) at aligned,
ragged and GEMV shapes, single and batched right-hand sides.
Tolerances: fp64 ≤ 1e-12 relative to the accumulated magnitude (sum |a||x|), fp32 ≤ 2e-5.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


def _glx():
    from glx import kernels
    return kernels


def _rel_err(got, ref, mag):
    return float((got.double() - ref).abs().max() / mag.clamp_min(1e-300).max())


SHAPES = [
    # (m, n, l)
    (256, 512, 2), (512, 1024, 16), (256, 512, 32), (1000, 1024, 32), (192, 4096, 16),
    (301, 517, 3), (333, 250, 17), (2048, 256, 1), (129, 64, 16), (64, 128, 32), (777, 640, 8),
    (4096, 8192, 16),
]


@pytest.mark.parametrize("dtype", ["f64", "f32"])
@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("variant", [0, 2, 3, 1820, 21820, 21410, 52224, 52228, 51328, 52324, 92278,
                                     92268, 92478])
def test_residual_and_gradient(shape, dtype, variant):
    k = _glx()
    m, n, l = shape
    dt = torch.float64 if dtype == "f64" else torch.float32
    g = torch.Generator(device="cuda").manual_seed(m * 7 + n * 3 + l)
    A = torch.randn(m, n, device="cuda", dtype=torch.float64, generator=g)
    X = torch.randn(n, l, device="cuda", dtype=torch.float64, generator=g)
    B = torch.randn(m, l, device="cuda", dtype=torch.float64, generator=g)
    Ad, Xd, Bd = A.to(dt), X.to(dt), B.to(dt)
    R, h = k.residual(Ad, Xd, Bd, variant=variant)
    torch.cuda.synchronize()
    ref = Ad.double() @ Xd.double() - Bd.double()
    mag = Ad.double().abs() @ Xd.double().abs() + Bd.double().abs()
    tol = 1e-13 if dtype == "f64" else 2e-6 * (n ** 0.5)
    assert _rel_err(R, ref, mag) < tol
    hr = 0.5 * float((R.double() ** 2).sum())
    # fp32: r*r rounds in fp32 (as NumPy does) before the fp64 sum
    assert abs(float(h.item()) - hr) <= (1e-12 if dtype == "f64" else 1e-6) * abs(hr) + 1e-300
    # A^T R with the exact R we just produced
    G = k.gradient(Ad, R)
    torch.cuda.synchronize()
    gref = Ad.double().T @ R.double()
    gmag = Ad.double().abs().T @ R.double().abs()
    tolg = 1e-13 if dtype == "f64" else 2e-6 * (m ** 0.5)
    assert _rel_err(G, gref, gmag) < tolg


@pytest.mark.parametrize("l", [16, 32])
def test_f32_dma_tile_default_plan(l, monkeypatch):
    """Round 4: f32 with one right-hand side and A beyond the Infinity Cache takes the LDS-DMA tile
    (92478, 64-column chunks) by default — C3's shape (the split-candidate dense pass A xc)."""
    monkeypatch.setenv("GLX_AX_DMA32", "1")
    k = _glx()
    m, n = 8192, 16384
    g = torch.Generator(device="cuda").manual_seed(l)
    A = torch.randn(m, n, device="cuda", dtype=torch.float32, generator=g)
    X = torch.randn(n, l, device="cuda", dtype=torch.float32, generator=g)
    B = torch.randn(m, l, device="cuda", dtype=torch.float32, generator=g)
    R, _ = k.residual(A, X, B)
    torch.cuda.synchronize()
    ref = A.double() @ X.double() - B.double()
    mag = A.double().abs() @ X.double().abs() + B.double().abs()
    assert _rel_err(R, ref, mag) < 2e-6 * (n ** 0.5)


BATCH_CODES = [0, 1420, 52224, 52324, 52228, 51328, 92278, 92268]


@pytest.mark.parametrize("dtype", ["f64", "f32"])
@pytest.mark.parametrize("shape", [(512, 1024, 32), (1000, 1024, 16), (129, 640, 32), (4096, 8192, 32)])
@pytest.mark.parametrize("nsrc", [2, 3])
@pytest.mark.parametrize("code", BATCH_CODES)
def test_residual_batch(monkeypatch, shape, dtype, nsrc, code):
    """A @ [X0 | X1 (| X2)] - B in one pass over A (GLX_AXB_VARIANT selects the batched tile)."""
    k = _glx()
    if code:
        monkeypatch.setenv("GLX_AXB_VARIANT", str(code))
    m, n, l = shape
    dt = torch.float64 if dtype == "f64" else torch.float32
    g = torch.Generator(device="cuda").manual_seed(m + n + l + nsrc)
    A = torch.randn(m, n, device="cuda", dtype=torch.float64, generator=g).to(dt)
    Xs = [torch.randn(n, l, device="cuda", dtype=torch.float64, generator=g).to(dt) for _ in range(nsrc)]
    B = torch.randn(m, l, device="cuda", dtype=torch.float64, generator=g).to(dt)
    Rs, sq = k.residual_batch(A, Xs, B)
    torch.cuda.synchronize()
    tol = 1e-13 if dtype == "f64" else 2e-6 * (n ** 0.5)
    for j, (R, X) in enumerate(zip(Rs, Xs)):
        ref = A.double() @ X.double() - B.double()
        mag = A.double().abs() @ X.double().abs() + B.double().abs()
        assert _rel_err(R, ref, mag) < tol, (j, code)
        s = float((R.double() ** 2).sum())
        assert abs(float(sq[j].item()) - s) <= (1e-12 if dtype == "f64" else 1e-6) * s


def test_mfma_layout_asymmetric():
    """A = I-like selector with an asymmetric X: catches row/col swaps in the MFMA C/D map."""
    k = _glx()
    for dt in (torch.float64, torch.float32):
        m, n, l = 64, 64, 32
        A = torch.eye(m, n, device="cuda", dtype=dt)
        X = (torch.arange(n * l, device="cuda", dtype=dt).reshape(n, l) * 3 + 1) % 251
        R, _ = k.residual(A, X, torch.zeros(m, l, device="cuda", dtype=dt))
        assert torch.equal(R, X)
        G = k.gradient(A, X)
        assert torch.equal(G, X)


def test_deterministic_repeat():
    k = _glx()
    A = torch.randn(1024, 2048, device="cuda", dtype=torch.float64)
    X = torch.randn(2048, 32, device="cuda", dtype=torch.float64)
    B = torch.randn(1024, 32, device="cuda", dtype=torch.float64)
    R1, h1 = k.residual(A, X, B)
    R2, h2 = k.residual(A, X, B)
    assert torch.equal(R1, R2) and torch.equal(h1, h2)
    assert torch.equal(k.gradient(A, R1), k.gradient(A, R1))


@pytest.mark.parametrize("l", [1, 2, 3, 8, 16, 17, 32, 64])
@pytest.mark.parametrize("dtype", ["f64", "f32"])
def test_prox_matches_reference_formula(l, dtype):
    """prox_th of gl_ProxGD_primal.py:65-71 including the (||w||<thres)+||w|| denominator."""
    k = _glx()
    dt = torch.float64 if dtype == "f64" else torch.float32
    npdt = np.float64 if dtype == "f64" else np.float32
    rng = np.random.default_rng(l)
    n = 1000
    W = rng.standard_normal((n, l)).astype(npdt)
    W[::7] *= 1e-4            # rows below thres take the quirky denominator
    W[::11] = 0               # all-zero rows
    t, mu, thres = 0.37, 0.02, 1e-3
    nrm = np.linalg.norm(W, axis=1).reshape(-1, 1)
    ref = W * np.clip(nrm - t * mu, a_min=0, a_max=None) / ((nrm < thres) + nrm)
    X, sums = k.prox(torch.from_numpy(W).cuda(), t, mu, thres)
    got = X.cpu().numpy()
    if dtype == "f64":
        np.testing.assert_allclose(got, ref, rtol=1e-14, atol=1e-300)
    else:
        np.testing.assert_allclose(got, ref, rtol=2e-6, atol=1e-30)
    s = sums.cpu().numpy()
    assert np.isclose(s[0], np.linalg.norm(ref.astype(np.float64), axis=1).sum(), rtol=1e-6 if dtype == "f32" else 1e-13)
    assert s[1] == np.abs(got).max()


def test_prox_nan_propagates():
    k = _glx()
    W = torch.ones(64, 4, device="cuda", dtype=torch.float64)
    W[5, 2] = float("nan")
    X, sums = k.prox(W, 0.1, 0.01)
    assert torch.isnan(X[5]).all()
    assert not torch.isnan(X[4]).any()
    assert np.isnan(sums[1].item())            # max|x| is NaN like np.max


@pytest.mark.parametrize("dtype", ["f64", "f32"])
@pytest.mark.parametrize("split", [1, 3, 8, 9, 17, 24, 33, 64])
def test_residual_batch_split_groups(monkeypatch, dtype, split):
    """Forced K splits: the finalize sums S slabs over G = 1..8 lanes (8 slabs per lane, ragged
    trailing lanes) and must give the same residual and sum of squares at every S."""
    k = _glx()
    monkeypatch.setenv("GLX_AXB_S", str(split))
    m, n, l = 1000, 8192, 32
    dt = torch.float64 if dtype == "f64" else torch.float32
    g = torch.Generator(device="cuda").manual_seed(split)
    A = torch.randn(m, n, device="cuda", dtype=torch.float64, generator=g).to(dt)
    Xs = [torch.randn(n, l, device="cuda", dtype=torch.float64, generator=g).to(dt) for _ in range(2)]
    B = torch.randn(m, l, device="cuda", dtype=torch.float64, generator=g).to(dt)
    Rs, sq = k.residual_batch(A, Xs, B)
    Rs2, sq2 = k.residual_batch(A, Xs, B)
    torch.cuda.synchronize()
    tol = 1e-13 if dtype == "f64" else 2e-6 * (n ** 0.5)
    for j, (R, X) in enumerate(zip(Rs, Xs)):
        ref = A.double() @ X.double() - B.double()
        mag = A.double().abs() @ X.double().abs() + B.double().abs()
        assert _rel_err(R, ref, mag) < tol, (j, split)
        s = float((R.double() ** 2).sum())
        assert abs(float(sq[j].item()) - s) <= (1e-12 if dtype == "f64" else 1e-6) * s
        assert torch.equal(R, Rs2[j]) and torch.equal(sq[j], sq2[j])   # deterministic


# A^T R tiles by code (NTL * 1000 + WL * 10 + PF; WL 2 = eight waves per panel, round 4),
# each against the fp64 reference, with K splits where the planner gives them
@pytest.mark.parametrize("dtype", ["f64", "f32"])
@pytest.mark.parametrize("shape", [(256, 512, 32), (512, 1024, 16), (1000, 1024, 32), (4096, 8192, 16),
                                   (8, 256, 32), (2052, 2048, 32)])
# the tiles the planner picks (round 6 pruned the measured-slower ones): f64 WL 0 PF 8 (+ non-
# temporal), f32 WL 1 PF 4 non-temporal, the eight-wave WL 2 panel, the f64 32-column panel WL 3
@pytest.mark.parametrize("code", [8, 1008, 1114, 1028, 38, 1038])
def test_gradient_atr_codes(monkeypatch, shape, dtype, code):
    monkeypatch.setenv("GLX_ATR_VARIANT", str(code))
    k = _glx()
    m, n, l = shape
    dt = torch.float64 if dtype == "f64" else torch.float32
    g = torch.Generator(device="cuda").manual_seed(m * 5 + n + l + code)
    A = torch.randn(m, n, device="cuda", dtype=torch.float64, generator=g).to(dt)
    R = torch.randn(m, l, device="cuda", dtype=torch.float64, generator=g).to(dt)
    G = k.gradient(A, R)
    torch.cuda.synchronize()
    gref = A.double().T @ R.double()
    gmag = A.double().abs().T @ R.double().abs()
    tolg = 1e-13 if dtype == "f64" else 2e-6 * (m ** 0.5)
    assert _rel_err(G, gref, gmag) < tolg
