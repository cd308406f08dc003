"""Whole-solve parity at the north-star size ("what's missing" item 2).

(m, n, l) = (8192, 16384, 32), fp64, the reference's ``gen_data`` instance (seed 97006855),
``opts = {"alpha0": 1/(sqrt(m)+sqrt(n))^2}``, every other option at the reference's default:
the HIP solver's whole continuation solve through the drop-in ``gl_<method>`` entry point
against the reference's own run of the same call (``tests/golden/ns_<method>.npz``, made by
``tests/golden/make_golden_ns.py`` importing ``/root/reference/code``). North-star bar:
identical k, fval and every f_hist / f_hist_best entry within 1e-8 relative, and the returned
iterate within 1e-6 of max|x|.
"""
import hashlib
import json
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.fixture(scope="module")
def instance():
    from oracle import numpy_ref
    meta = json.load(open(os.path.join(GOLD, "ns_gl_ProxGD_primal.json")))
    m, n, l = meta["m"], meta["n"], meta["l"]
    A, _, u, x0, mu = numpy_ref.gen_data(m, n, l, meta["seed"])
    b = np.load(os.path.join(GOLD, "ns_instance_b.npz"))["b"]
    assert _sha(A) == meta["sha256"]["A"] and _sha(x0) == meta["sha256"]["x0"]
    assert _sha(u) == meta["sha256"]["u"] and _sha(b) == meta["sha256"]["b"]
    At = torch.from_numpy(A).cuda()
    del A
    return At, torch.from_numpy(b).cuda(), x0, mu, meta["opts"]


@pytest.mark.parametrize("method", ["gl_ProxGD_primal", "gl_FProxGD_primal"])
def test_whole_solve_north_star_size(instance, method):
    import importlib
    At, bt, x0, mu, opts = instance
    gold = np.load(os.path.join(GOLD, "ns_%s.npz" % method))
    fn = getattr(importlib.import_module(method), method)
    x, k, out = fn(torch.from_numpy(x0).cuda(), At, bt, mu, dict(opts))
    torch.cuda.synchronize()
    x = x.cpu().numpy() if hasattr(x, "cpu") else np.asarray(x)
    assert k == int(gold["k"]), (k, int(gold["k"]))
    fg = float(gold["fval"])
    assert abs(float(out["fval"]) - fg) <= 1e-8 * abs(fg), (float(out["fval"]), fg)
    for key in ("f_hist", "f_hist_best"):
        got = np.asarray([float(v) for v in out[key]])
        ref = gold[key]
        assert got.shape == ref.shape
        rel = np.max(np.abs(got - ref) / np.abs(ref))
        assert rel <= 1e-8, (key, rel, int(np.argmax(np.abs(got - ref) / np.abs(ref))))
    xr = gold["x"].astype(np.float64)
    assert np.max(np.abs(x - xr)) <= 1e-6 * np.max(np.abs(xr))


# C3's default path (round 6: the dense [xc | y_next] batch again) ends at this
# objective, bit for bit run to run (every kernel's order is fixed): the tripwire below
# (profiles/r5_d/c3_band.jsonl, variant "dense").
C3_DEFAULT_FVAL = 124.66799582996916


def test_whole_solve_c3_fp32():
    """BASELINE config C3: gl_FProxGD_primal in fp32 at (8192, 16384, 32), the whole continuation
    solve against the reference's own fp32 run of the same call (tests/golden/make_golden_c3.py)
    and its fp64 run (ns_gl_FProxGD_primal).

    The C3 solve stops at maxit (4500, not converged), so its fp32 objective depends on the
    summation order: eleven equally valid orders end 3.4e-7 .. 8.9e-5 from the reference's fp32
    objective, every one 7.0e-3 .. 7.1e-3 from the fp64 objective, as the reference's own fp32 run
    is (scripts/c3_band.py, profiles/r5_d/c3_band.jsonl). The default path is the order that meets
    the fp32 bar of SURVEY §8d (the bar is not widened to fit a default):
      - fval within 1e-6 of the reference's fp32 run (measured 3.4e-7);
      - fval within 1e-2 of the reference's fp64 run (the fp32 arithmetic's own distance, 7e-3);
      - k within 0.5 % (measured identical, 4500 = maxit); where k agrees, every f_hist entry
        within 5e-3 and x within 5e-2 of max|x| (mid-solve drift of two fp32 implementations,
        up to 1.8e-3 / 3.0e-2, profiles/r4_c3gold/);
      - tripwire: the default path's objective equals C3_DEFAULT_FVAL to 1e-12 — it pins the
        default kernels' summation order; a change of any fp32 order on this path must be
        re-checked against the 1e-6 bar before it is re-recorded."""
    import importlib
    meta_path = os.path.join(GOLD, "c3_gl_FProxGD_primal.json")
    if not os.path.exists(meta_path):
        pytest.skip("C3 fixture not generated")
    meta = json.load(open(meta_path))
    from oracle import numpy_ref
    m, n, l = meta["m"], meta["n"], meta["l"]
    A, _, u, x0, mu = numpy_ref.gen_data(m, n, l, meta["seed"])
    b = np.load(os.path.join(GOLD, "ns_instance_b.npz"))["b"]
    A32, b32, x032 = (a.astype(np.float32) for a in (A, b, x0))
    del A
    assert _sha(A32) == meta["sha256"]["A32"] and _sha(b32) == meta["sha256"]["b32"]
    assert _sha(x032) == meta["sha256"]["x032"]
    gold = np.load(os.path.join(GOLD, "c3_gl_FProxGD_primal.npz"))
    gold64 = float(np.load(os.path.join(GOLD, "ns_gl_FProxGD_primal.npz"))["fval"])
    fn = getattr(importlib.import_module("gl_FProxGD_primal"), "gl_FProxGD_primal")
    x, k, out = fn(torch.from_numpy(x032).cuda(), torch.from_numpy(A32).cuda(),
                   torch.from_numpy(b32).cuda(), mu, dict(meta["opts"]))
    torch.cuda.synchronize()
    kg = int(gold["k"])
    assert abs(k - kg) <= max(1, int(0.005 * kg)), (k, kg)
    fg, fv = float(gold["fval"]), float(out["fval"])
    assert abs(fv - fg) <= 1e-6 * abs(fg), (fv, fg)
    assert abs(fv - gold64) <= 1e-2 * abs(gold64), (fv, gold64)
    if k == kg:
        got = np.asarray([float(v) for v in out["f_hist"]])
        rel = np.max(np.abs(got - gold["f_hist"]) / np.abs(gold["f_hist"]))
        assert rel <= 5e-3, rel
        xr = gold["x"].astype(np.float64)
        xx = x.cpu().numpy().astype(np.float64) if hasattr(x, "cpu") else np.asarray(x, np.float64)
        assert np.max(np.abs(xx - xr)) <= 5e-2 * np.max(np.abs(xr))
    assert abs(fv - C3_DEFAULT_FVAL) <= 1e-12 * abs(C3_DEFAULT_FVAL), (fv, C3_DEFAULT_FVAL)


@pytest.mark.parametrize("tag,method", [("c2", "gl_ProxGD_primal"), ("c4", "gl_SGD_primal")])
def test_whole_solve_baseline_configs(tag, method):
    """BASELINE configs C2 (gl_ProxGD_primal fp64, (4096, 8192, 16)) and C4 (gl_SGD_primal fp64,
    l = 1, (65536, 8192)): the whole solve against the reference's own run of the same call
    (tests/golden/make_golden_<tag>.py). North-star fp64 bar: identical k, fval and every
    f_hist / f_hist_best entry within 1e-8 relative, the iterate within 1e-6 of max|x|."""
    import importlib
    gdir = GOLD
    meta_path = os.path.join(gdir, "%s_%s.json" % (tag, method))
    if not os.path.exists(meta_path):
        pytest.skip("%s fixture not in %s" % (tag, gdir))
    meta = json.load(open(meta_path))
    from oracle import numpy_ref
    A, _, u, x0, mu = numpy_ref.gen_data(meta["m"], meta["n"], meta["l"], meta["seed"])
    gold = np.load(os.path.join(gdir, "%s_%s.npz" % (tag, method)))
    b = gold["b"]
    assert _sha(A) == meta["sha256"]["A"] and _sha(x0) == meta["sha256"]["x0"]
    assert _sha(u) == meta["sha256"]["u"] and _sha(b) == meta["sha256"]["b"]
    fn = getattr(importlib.import_module(method), method)
    At = torch.from_numpy(A).cuda()
    del A
    x, k, out = fn(torch.from_numpy(x0).cuda(), At, torch.from_numpy(b).cuda(), mu, dict(meta["opts"]))
    torch.cuda.synchronize()
    x = x.cpu().numpy()
    assert k == int(gold["k"]), (k, int(gold["k"]))
    fg = float(gold["fval"])
    assert abs(float(out["fval"]) - fg) <= 1e-8 * abs(fg), (float(out["fval"]), fg)
    for key in ("f_hist", "f_hist_best"):
        got = np.asarray([float(v) for v in out[key]])
        rel = np.max(np.abs(got - gold[key]) / np.abs(gold[key]))
        assert rel <= 1e-8, (key, rel)
    xr = gold["x"].astype(np.float64)
    assert np.max(np.abs(x - xr)) <= 1e-6 * np.max(np.abs(xr))
