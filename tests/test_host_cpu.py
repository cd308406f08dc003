"""CPU-only checks of the native library's host surface and the Python boundary.

No GPU is touched: the library loads (linked against torch's HIP runtime), exports every
symbol include/glx.h declares, its struct layouts agree with the ctypes mirror, and the
host-side logic (option merging, workspace planning, shard ranges) behaves.
"""
import ctypes
import os
import re
import subprocess
import tempfile

import pytest

from conftest import ROOT


def test_library_loads_and_exports_header_symbols():
    from glx import _lib
    h = _lib.lib()
    header = open(os.path.join(ROOT, "include", "glx.h")).read()
    declared = set(re.findall(r"\b(glx_[a-z_0-9]+)\s*\(", header))
    assert declared, "no declarations parsed"
    for name in sorted(declared):
        assert hasattr(h, name), name
    assert set(_lib.EXPORTED) == declared
    assert h.glx_abi_version() == 2


def test_single_hip_runtime_in_process():
    import torch  # noqa: F401
    from glx import _lib
    _lib.lib()
    maps = open("/proc/self/maps").read()
    runtimes = set(re.findall(r"(\S*libamdhip64\S*)", maps))
    assert len(runtimes) == 1, runtimes


def test_struct_layout_matches_c():
    """Compile a tiny C program against include/glx.h and compare sizeof/offsetof."""
    from glx import _lib
    src = r'''
#include <stdio.h>
#include <stddef.h>
#include "glx.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu %zu\n", sizeof(glx_opts), sizeof(glx_problem),
         sizeof(glx_result), offsetof(glx_opts, max_total_iters), offsetof(glx_problem, mu0),
         offsetof(glx_result, syncs), offsetof(glx_opts, ax_variant), offsetof(glx_opts, split_cand),
         offsetof(glx_opts, dc_window), offsetof(glx_result, record_waits));
  return 0;
}'''
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        exe = os.path.join(d, "t")
        open(c, "w").write(src)
        subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe], check=True)
        got = [int(v) for v in subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split()]
    want = [ctypes.sizeof(_lib.GlxOpts), ctypes.sizeof(_lib.GlxProblem), ctypes.sizeof(_lib.GlxResult),
            _lib.GlxOpts.max_total_iters.offset, _lib.GlxProblem.mu0.offset, _lib.GlxResult.syncs.offset,
            _lib.GlxOpts.ax_variant.offset, _lib.GlxOpts.split_cand.offset,
            _lib.GlxOpts.dc_window.offset, _lib.GlxResult.record_waits.offset]
    assert got == want


def test_default_opts_match_reference_tables():
    from glx import _lib
    from oracle import numpy_ref
    o = _lib.default_opts(_lib.GLX_PROXGD)
    d = numpy_ref.PROXGD_DEFAULTS
    assert (o.maxit, o.thres, o.alpha0, o.ftol, o.stable_len_threshold, o.ls_coeff, o.ls_maxit) == \
        (d["maxit"], d["thres"], d["alpha0"], d["ftol"], d["stable_len_threshold"],
         d["line_search_attenuation_coeffi"], d["maxit_line_search_iter"])
    o = _lib.default_opts(_lib.GLX_FPROXGD)
    d = numpy_ref.FPROXGD_DEFAULTS
    assert (o.maxit, o.alpha0, o.ls_coeff) == (d["maxit"], d["alpha0"], d["line_search_attenuation_coeffi"])
    o = _lib.default_opts(_lib.GLX_SGD)
    d = numpy_ref.SGD_DEFAULTS
    assert (o.maxit, o.alpha0, o.ftol, o.step_type) == (d["maxit"], d["alpha0"], d["ftol"], _lib.STEP_TYPES["diminishing"])
    o = _lib.default_opts(_lib.GLX_GD)
    assert (o.maxit, o.delta) == (numpy_ref.GD_DEFAULTS["maxit"], numpy_ref.GD_DEFAULTS["delta"])
    o = _lib.default_opts(_lib.GLX_FGD)
    assert (o.maxit, o.delta, o.ls_coeff) == (1500, 1e-6, 0.98)


def test_make_opts_merging_and_errors():
    from glx import _lib
    from glx.solver import make_opts
    user = {"maxit": 7, "alpha0": 0.5, "unknown_key": 1, "line_search_attenuation_coeffi": 0.5,
            "exact_objective": True}
    o = make_opts(_lib.GLX_PROXGD, user)
    assert (o.maxit, o.alpha0, o.ls_coeff, o.exact_objective, o.ftol) == (7, 0.5, 0.5, 1, 1e-6)
    assert user["maxit"] == 7 and "unknown_key" in user
    with pytest.raises(ValueError):
        make_opts(_lib.GLX_PROXGD, {"step_type": "nope"})
    with pytest.raises(ValueError):
        make_opts(_lib.GLX_SGD, {"step_type": "line_search"})


def test_workspace_planning_host_only():
    from glx import _lib
    from glx.solver import make_opts
    for meth in (_lib.GLX_PROXGD, _lib.GLX_FPROXGD):
        for (m, n, l, dt) in [(8192, 16384, 32, 1), (4096, 8192, 16, 1), (65536, 8192, 1, 1),
                              (256, 512, 2, 1), (301, 517, 3, 0), (8192, 16384, 32, 0)]:
            p = _lib.GlxProblem(dtype=dt, method=meth, m=m, n=n, l=l, A=256, b=256, x=256, mu0=0.01)
            nb = ctypes.c_size_t(0)
            _lib.check(_lib.lib().glx_workspace_bytes(ctypes.byref(p), ctypes.byref(make_opts(meth, {})),
                                                      ctypes.byref(nb)))
            es = 8 if dt == 1 else 4
            # split-candidate trials (m n * 8 B of 768 MiB or more; fp64 only by default — fp32
            # FProxGD's split form is opt-in, GLX_SPLIT_F32=1, round 6) keep a transposed copy of A
            # (kernels_gather.hip); FProxGD's also e_c and three A thr(x) residual-sized slots
            gate = (64 if meth == _lib.GLX_PROXGD and l == 32 else 768) * 2**20   # kSplitMinBytes*
            split = dt == 1 and l in (16, 32) and m * n * 8 >= gate
            at = es * m * n if split else 0
            extra = es * (n * l + 3 * m * l) if (split and meth == _lib.GLX_FPROXGD) else 0
            assert nb.value >= es * (2 * n * l + 2 * m * l) + at + extra  # x-buffers + residuals at least
            assert nb.value < at + es * (m * n) // 4 + (64 << 20)   # else never close to the size of A


def test_invalid_problem_rejected_on_host():
    from glx import _lib
    from glx.solver import make_opts
    p = _lib.GlxProblem(dtype=1, method=0, m=8, n=8, l=500, A=256, b=256, x=256, mu0=0.01)
    nb = ctypes.c_size_t(0)
    rc = _lib.lib().glx_workspace_bytes(ctypes.byref(p), ctypes.byref(make_opts(0, {})), ctypes.byref(nb))
    assert rc != 0 and b"128" in _lib.lib().glx_last_error()
    p = _lib.GlxProblem(dtype=1, method=0, m=8, n=8, l=2, A=255, b=256, x=256, mu0=0.01)
    assert _lib.lib().glx_workspace_bytes(ctypes.byref(p), ctypes.byref(make_opts(0, {})), ctypes.byref(nb)) != 0


def test_product_path_has_no_cpu_fallback(monkeypatch):
    import torch
    from glx import solver
    monkeypatch.setattr(torch.cuda, "is_available", lambda: False)
    import numpy as np
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        solver.solve("gl_ProxGD_primal", np.zeros((4, 2)), np.zeros((3, 4)), np.zeros((3, 2)), 1e-2, {})


def test_shard_rows_partition():
    from glx.dist import shard_rows
    for m in (1, 7, 8192, 131072, 1000003):
        for w in (1, 2, 3, 8):
            if m < w:
                continue
            ranges = [shard_rows(m, w, r) for r in range(w)]
            assert ranges[0][0] == 0 and ranges[-1][1] == m
            assert all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))
            sizes = [b - a for a, b in ranges]
            assert max(sizes) - min(sizes) <= 1


def test_plan_describe_picks_tiles_by_shape():
    """The planner (host code) picks MFMA tiles for l = 16/32 and VALU for other l."""
    from glx import _lib
    ns = _lib.plan_describe(_lib.GLX_F64, 8192, 16384, 32)
    assert "ax2=k_ax_lds<" in ns and "atr=k_atr_mfma<" in ns, ns
    gemv = _lib.plan_describe(_lib.GLX_F64, 65536, 8192, 1)
    assert "k_ax_valu" in gemv and "k_atr_valu" in gemv, gemv
    # n not a multiple of the LDS chunk: falls back to a register tile, never an invalid one
    odd = _lib.plan_describe(_lib.GLX_F64, 1000, 1000, 32)
    assert "ax2=" in odd and "ax3=" in odd, odd
    with pytest.raises(_lib.GlxError):
        _lib.plan_describe(_lib.GLX_F64, 0, 16, 16)


def test_kernel_workspace_covers_every_planned_split():
    """glx_kernel_workspace_bytes must hold the partial slabs of the largest K split any tile
    (single or batched, register or LDS) plans, else the single-kernel calls refuse to run."""
    from glx import _lib
    for shp in [(512, 1024, 16), (512, 1024, 32), (4096, 8192, 16), (129, 640, 32)]:
        nb = ctypes.c_size_t(0)
        _lib.check(_lib.lib().glx_kernel_workspace_bytes(_lib.GLX_F64, *shp, ctypes.byref(nb)))
        splits = [int(s) for s in re.findall(r"S=(\d+)", _lib.plan_describe(_lib.GLX_F64, *shp))]
        m, n, l = shp
        assert nb.value >= 8 * m * l * max(splits) * 3, (shp, nb.value, splits)
