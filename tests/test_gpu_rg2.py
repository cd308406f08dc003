"""The l = 16 one-pass trial batch + gradient (kernels_rg2.hip, SURVEY §8f row 1 at C2's width):
R0 = A X0 - B, R1 = A X1 - B and G = A^T R1 from ONE read of A (reference
gl_ProxGD_primal.py:89-92 and :112 `A @ z`, `A @ p_thr`, :129 the gradient at the candidate),
against an fp64 torch reference of the same products. Tolerance 1e-13 relative to the accumulated
magnitude (sum |a||x| + |b| for R, sum |a||r| for G), as the two-pass kernel tests; every sum has a
fixed order, so two calls agree bit for bit.
"""
import os
import subprocess
import sys

import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rel(got, ref, mag):
    return float((got - ref).abs().max() / mag.clamp_min(1e-300).max())


# (m, n): P = n / 256 panels (a power of two, 2..128), RG = 256 / P row groups, m a multiple of
# 64 RG (NB = m / RG / 16 blocks per group, a multiple of the A-waves' 4 tile buffers).
# (4096, 8192) is SURVEY's C2 (RG = 8: the XCD-local hand-off).
SHAPES = [(4096, 8192), (4096, 2048), (16384, 512), (2048, 32768), (8192, 4096), (512, 16384)]


def _inputs(m, n, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    A = torch.randn(m, n, device="cuda", dtype=torch.float64, generator=g)
    X0 = torch.randn(n, 16, device="cuda", dtype=torch.float64, generator=g)
    X1 = torch.randn(n, 16, device="cuda", dtype=torch.float64, generator=g)
    B = torch.randn(m, 16, device="cuda", dtype=torch.float64, generator=g)
    return A, X0, X1, B


def _check(m, n, expect_one_pass=True):
    from glx import kernels
    A, X0, X1, B = _inputs(m, n, m + 5 * n)
    R0, R1, G, ran = kernels.residual_gradient2(A, X0, X1, B, one_pass=True)
    torch.cuda.synchronize()
    assert ran == expect_one_pass
    assert torch.isfinite(G).all()
    assert _rel(R0, A @ X0 - B, A.abs() @ X0.abs() + B.abs()) < 1e-13
    assert _rel(R1, A @ X1 - B, A.abs() @ X1.abs() + B.abs()) < 1e-13
    assert _rel(G, A.T @ R1, A.abs().T @ R1.abs()) < 1e-13   # the gradient of the R1 produced
    return A, X0, X1, B, R0, R1, G


@pytest.mark.parametrize("shape", SHAPES)
def test_rg2_matches_fp64(shape):
    from glx import kernels
    A, X0, X1, B, R0, R1, G = _check(*shape)
    for _ in range(2):   # repeated launches on fresh workspaces: identical bits
        S0, S1, G2, ran = kernels.residual_gradient2(A, X0, X1, B, one_pass=True)
        assert ran and torch.equal(R0, S0) and torch.equal(R1, S1) and torch.equal(G, G2)


def test_rg2_residuals_match_two_pass_bits():
    """The residuals are A @ X's fixed-order sums minus B; the two-pass path (one_pass=0) agrees
    with the one-pass kernel's R within rounding and its G within the tolerance."""
    from glx import kernels
    A, X0, X1, B = _inputs(4096, 8192, 7)
    R0, R1, G, ran = kernels.residual_gradient2(A, X0, X1, B, one_pass=True)
    T0, T1, TG, tran = kernels.residual_gradient2(A, X0, X1, B, one_pass=False)
    assert ran and not tran
    assert _rel(R0, T0, A.abs() @ X0.abs() + B.abs()) < 1e-13
    assert _rel(R1, T1, A.abs() @ X1.abs() + B.abs()) < 1e-13
    assert _rel(G, TG, A.abs().T @ R1.abs()) < 1e-13


def test_rg2_unsupported_shapes_run_two_passes():
    from glx import kernels
    # ragged m, n % 256, P = 24, NB = 2
    for m, n in [(1000, 8192), (4096, 8448), (4096, 6144), (1024, 2048)]:
        A, X0, X1, B = _inputs(m, n, m + n)
        R0, R1, G, ran = kernels.residual_gradient2(A, X0, X1, B, one_pass=True)
        assert not ran
        assert _rel(R1, A @ X1 - B, A.abs() @ X1.abs() + B.abs()) < 1e-13
        assert _rel(G, A.T @ R1, A.abs().T @ R1.abs()) < 1e-13


def _check_forced_timeout():
    """Every hand-off wait gives up at once (GLX_RG_SPIN=0): the kernel flags the error, the host
    recomputes with two passes and reports that the one-pass result was not used."""
    _check(4096, 8192, expect_one_pass=False)


def test_rg2_timeout_falls_back():
    code = "import sys; sys.path.insert(0, %r); import tests.test_gpu_rg2 as t; t._check_forced_timeout()" % ROOT
    env = dict(os.environ, GLX_RG_SPIN="0",
               PYTHONPATH=os.pathsep.join([ROOT, os.path.join(ROOT, "convex-optimization_amd")]))
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=100)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
