"""The split-candidate trial's flagged-row product A e (round 5, kernels_gather.hip k_at_rows).

Reference: the line-search candidate's objective g(p) = 1/2 ||A p - b||^2 (gl_ProxGD_primal.py:91,
:112) with p = p_thr + e, e = p - p_thr nonzero only where the hard threshold (:127) zeroed an
entry; FProxGD's A y_next from A e_c (gl_FProxGD_primal.py:92-97, :136). libglx computes A e from a
transposed copy At = A^T over the flagged rows only. Checked here through the C ABI
(glx_flagged_rows_product) against an fp64 torch reference of the same product, in its three forms
(the MFMA row form, the VALU column-list gather of rounds 2-4, and the round-5 bitmap gather that
builds the same lists in LDS: bit-identical to the list form), on aligned, large, ragged and
empty flag sets, and bit-reproducible run to run.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


def _case(m, n, l, frac, dtype, seed, dense_rows=False, garbage=False):
    g = torch.Generator(device="cpu").manual_seed(seed)
    At = torch.randn(n, m, generator=g, dtype=torch.float64)
    E = torch.zeros(n, l, dtype=torch.float64)
    flagged = torch.rand(n, generator=g) < frac
    rows = flagged.nonzero().flatten()
    if dense_rows:            # FISTA's e_c: whole small rows
        E[rows] = 1e-4 * torch.randn(len(rows), l, generator=g, dtype=torch.float64)
    else:                     # ProxGD's e: about one entry per flagged row
        cols = torch.randint(0, l, (len(rows),), generator=g)
        E[rows, cols] = 1e-4 * torch.randn(len(rows), generator=g, dtype=torch.float64)
        extra = rows[torch.rand(len(rows), generator=g) < 0.1]
        E[extra, (cols[:len(extra)] + 1) % l] = 3e-4
    masks = torch.zeros(n + 64, dtype=torch.int64)
    nz = (E != 0)
    w = (nz.to(torch.int64) << torch.arange(l, dtype=torch.int64)).sum(1)
    masks[:n] = w
    Eg = E.clone()
    if garbage:               # values in unflagged rows must be ignored by the row form
        unfl = (~nz.any(1)).nonzero().flatten()[:7]
        Eg[unfl] = 5.0
    ref = At[nz.any(1)].T @ E[nz.any(1)]
    # masks as uint32 bit patterns in an int32 tensor (bit 31 may be set at l = 32)
    m32 = torch.from_numpy(masks.numpy().astype(np.uint32).view(np.int32))
    return (At.to(dtype).cuda(), Eg.to(dtype).cuda(), m32.cuda(), ref,
            At.abs().T @ E.abs())


@pytest.mark.parametrize("m,n,l,frac,dense", [
    (8192, 16384, 32, 0.2, False),     # north-star size, ProxGD-like e (~3 300 flagged rows)
    (8192, 16384, 32, 0.45, True),     # FISTA-like e_c, dense flagged rows
    (4096, 8192, 16, 0.25, False),     # C2's shape
    (256, 512, 32, 0.5, True),
    (1024, 2048, 16, 0.0, False),      # nothing flagged
    (192, 300, 32, 0.3, True),         # ragged n (K ranges cut at 64-row chunks)
])
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_flagged_rows_product_vs_torch(m, n, l, frac, dense, dtype):
    from glx import kernels
    At, E, masks, ref, scale = _case(m, n, l, frac, dtype, seed=m + n + l, dense_rows=dense)
    tol = 1e-13 if dtype == torch.float64 else 2e-6
    Ys = {}
    for form in (0, 1, 2):
        Ys[form] = kernels.flagged_rows_product(At, E, masks, form=form)
        Y = Ys[form].double().cpu()
        err = (Y - ref).abs().max().item()
        bound = tol * max(1.0, scale.max().item())
        assert err <= bound, (form, err, bound)
    # the bitmap gather walks the same ascending lists as k_e_lists + k_at_gather: bit-identical
    assert torch.equal(Ys[1], Ys[2])


def test_row_form_ignores_unflagged_rows():
    from glx import kernels
    At, E, masks, ref, scale = _case(512, 1024, 32, 0.3, torch.float64, seed=5, dense_rows=True,
                                     garbage=True)
    Y = kernels.flagged_rows_product(At, E, masks, form=0).cpu()
    assert (Y - ref).abs().max().item() <= 1e-13 * scale.max().item()


def test_row_form_bit_reproducible():
    from glx import kernels
    At, E, masks, ref, _ = _case(8192, 16384, 32, 0.3, torch.float64, seed=9, dense_rows=True)
    Y0 = kernels.flagged_rows_product(At, E, masks, form=0)
    for _ in range(3):
        assert torch.equal(kernels.flagged_rows_product(At, E, masks, form=0), Y0)


def test_row_form_needs_whole_panels():
    from glx import kernels
    from glx._lib import GlxError
    At, E, masks, ref, _ = _case(100, 256, 16, 0.3, torch.float64, seed=3)
    with pytest.raises(GlxError):
        kernels.flagged_rows_product(At, E, masks, form=0)
    for form in (1, 2):   # the gathers take any m
        Y = kernels.flagged_rows_product(At, E, masks, form=form).cpu()
        assert (Y - ref).abs().max().item() <= 1e-12


@pytest.mark.parametrize("variant", ["16,256,0", "8,128,0", "16,128,0", "8,256,1", "16,256,1", "8,128,1"])
def test_bitmap_gather_variants_bit_identical(variant, monkeypatch):
    """GLX_GATHER_BM = loads in flight, bitmap words per segment, 16-B row form: none changes a
    row's summation order, so every variant equals the default bit for bit (fp64 and fp32)."""
    from glx import kernels
    for dtype in (torch.float64, torch.float32):
        At, E, masks, ref, _ = _case(4096, 16384, 32, 0.2, dtype, seed=17)
        monkeypatch.delenv("GLX_GATHER_BM", raising=False)
        Y0 = kernels.flagged_rows_product(At, E, masks, form=2)
        monkeypatch.setenv("GLX_GATHER_BM", variant)
        Y1 = kernels.flagged_rows_product(At, E, masks, form=2)
        assert torch.equal(Y0, Y1), (variant, dtype)
