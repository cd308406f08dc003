"""The fused residual-gradient pass (kernels_fused.hip): R = A X - B and
G = A^T R from ONE read of A, against an fp64 torch reference of the same two products
(reference gl_ProxGD_primal.py:129). Tolerance 1e-13 relative to the accumulated magnitude
(sum |a||x| for R, sum |a||r| for G), as the kernel-level tests of the two-pass path; the sums
are deterministic (fixed-order exchange), so two calls agree bit for bit.
"""
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


def _rel(got, ref, mag):
    return float((got - ref).abs().max() / mag.clamp_min(1e-300).max())


# (m, n): row groups RG = 256 / (n / 512), m a multiple of 16 RG with >= 2 blocks per group
SHAPES = [(8192, 16384), (1024, 4096), (2048, 8192), (4096, 16384), (1024, 16384), (65536, 1024)]


@pytest.mark.parametrize("xcd", ["1", "0"])
@pytest.mark.parametrize("shape", SHAPES)
def test_resgrad_matches_fp64(shape, xcd, monkeypatch):
    # xcd "1": row groups = the XCDs (HW_REG_XCC_ID) where there are 8 of them, XCD-local
    # exchange; "0": the placement-independent sc1 exchange. Read once per process, so the
    # "0" cases run in a child process.
    if xcd == "0":
        import subprocess, sys, os
        code = ("import os, sys; sys.path.insert(0, %r); os.environ['GLX_RG_XCD'] = '0'; "
                "import tests.test_gpu_resgrad as t; t._check(%d, %d)" % (
                    os.path.dirname(os.path.dirname(os.path.abspath(__file__))), shape[0], shape[1]))
        env = dict(os.environ, GLX_RG_XCD="0",
                   PYTHONPATH=os.pathsep.join([os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                               os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                            "convex-optimization_amd")]))
        p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=100)
        assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
        return
    _check(*shape)


def _check(m, n):
    from glx import kernels
    l = 32
    g = torch.Generator(device="cuda").manual_seed(m + 3 * n)
    A = torch.randn(m, n, device="cuda", dtype=torch.float64, generator=g)
    X = torch.randn(n, l, device="cuda", dtype=torch.float64, generator=g)
    B = torch.randn(m, l, device="cuda", dtype=torch.float64, generator=g)
    R, G, fused = kernels.residual_gradient(A, X, B, one_pass=True)
    torch.cuda.synchronize()
    assert fused, "the one-pass kernel did not run for a supported shape"
    Rr = A @ X - B
    Gr = A.T @ R          # the gradient of the residual the kernel produced
    assert torch.isfinite(G).all()
    assert _rel(R, Rr, A.abs() @ X.abs() + B.abs()) < 1e-13
    assert _rel(G, Gr, A.abs().T @ R.abs()) < 1e-13
    R2, G2, _ = kernels.residual_gradient(A, X, B, one_pass=True)
    assert torch.equal(R, R2) and torch.equal(G, G2)


def test_resgrad_unsupported_shape_falls_back():
    from glx import kernels
    m, n, l = 1000, 1024, 16
    A = torch.randn(m, n, device="cuda", dtype=torch.float64)
    X = torch.randn(n, l, device="cuda", dtype=torch.float64)
    B = torch.randn(m, l, device="cuda", dtype=torch.float64)
    R, G, fused = kernels.residual_gradient(A, X, B, one_pass=True)
    assert not fused
    # a supported shape runs two passes unless one_pass is asked for
    A2 = torch.randn(1024, 4096, device="cuda", dtype=torch.float64)
    X2 = torch.randn(4096, 32, device="cuda", dtype=torch.float64)
    B2 = torch.randn(1024, 32, device="cuda", dtype=torch.float64)
    R3, G3, f3 = kernels.residual_gradient(A2, X2, B2)
    assert not f3
    assert _rel(G3, A2.T @ R3, A2.abs().T @ R3.abs()) < 1e-13
    assert _rel(R, A @ X - B, A.abs() @ X.abs() + B.abs()) < 1e-13
    assert _rel(G, A.T @ R, A.abs().T @ R.abs()) < 1e-13


def _check_forced_timeout(m, n):
    """Every hand-off wait gives up at once (GLX_RG_SPIN=0): the kernel flags the error, the host
    reads it back and recomputes R and G with two passes, and reports that the one-pass kernel's
    result was not used."""
    from glx import kernels
    l = 32
    g = torch.Generator(device="cuda").manual_seed(m + n)
    A = torch.randn(m, n, device="cuda", dtype=torch.float64, generator=g)
    X = torch.randn(n, l, device="cuda", dtype=torch.float64, generator=g)
    B = torch.randn(m, l, device="cuda", dtype=torch.float64, generator=g)
    R, G, fused = kernels.residual_gradient(A, X, B, one_pass=True)
    torch.cuda.synchronize()
    assert not fused, "a timed-out one-pass result was reported as used"
    assert _rel(R, A @ X - B, A.abs() @ X.abs() + B.abs()) < 1e-13
    assert _rel(G, A.T @ R, A.abs().T @ R.abs()) < 1e-13


@pytest.mark.parametrize("xcd", ["1", "0"])
def test_resgrad_timeout_falls_back(xcd):
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys; sys.path.insert(0, %r); import tests.test_gpu_resgrad as t; "
            "t._check_forced_timeout(8192, 16384)" % root)
    env = dict(os.environ, GLX_RG_SPIN="0", GLX_RG_XCD=xcd,
               PYTHONPATH=os.pathsep.join([root, os.path.join(root, "convex-optimization_amd")]))
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=100)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
