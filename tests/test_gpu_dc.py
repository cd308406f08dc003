"""Device-controlled ProxGD batches (solver.cpp dc_run, kernels_elem.hip
ctl_decide).

In the speculative steady state the Armijo test (code/gl_ProxGD_primal.py:89-92), the next
record and the stop rule (:118-125) run on the device, in the last block of the trial's
residual finalize, and the host keeps up to GLX_DC_BATCH iterations queued. The decision
arithmetic is the host's term for term, so every run must be bit-identical to host control
(GLX_DC_BATCH=0): same k, same f_hist to the last bit, same iterate. Covered: accepted-only
stretches ending at the stop rule and at maxit, rejections (alpha0 = 2.5x the safe step) that
cancel the queued work, the split-candidate gather form, fp32, and run() called in short
slices (the batch budget follows run()'s step limit).
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


def _instance(m, n, l, seed=2024):
    from oracle import numpy_ref
    A, b, u, x0, mu = numpy_ref.gen_data(m, n, l, seed)
    return A, b, x0, mu, numpy_ref.step_size_for(m, n)


def _run(monkeypatch, window, shape, dtype=np.float64, alpha_scale=1.0, opts=None, slices=0,
         env=None, method="gl_ProxGD_primal"):
    import glx
    monkeypatch.setenv("GLX_DC_BATCH", str(window))
    for k, v in (env or {}).items():
        monkeypatch.setenv(k, v)
    A, b, x0, mu, alpha0 = _instance(*shape)
    o = {"alpha0": alpha0 * alpha_scale}
    o.update(opts or {})
    At, bt, xt = (torch.from_numpy(a.astype(dtype)).cuda() for a in (A, b, x0))
    s = glx.Session(method, xt, At, bt, mu, o)
    if slices:
        while not s.finished:
            s.run(slices)
    else:
        s.run(0)
    res = s.finish()
    s.close()
    torch.cuda.synchronize()
    return xt.cpu().numpy(), res


def _same(a, b):
    (x_a, r_a), (x_b, r_b) = a, b
    assert r_a["k"] == r_b["k"]
    assert np.array_equal(np.asarray(r_a["f_hist"]), np.asarray(r_b["f_hist"]))
    assert r_a["fval"] == r_b["fval"]
    assert np.array_equal(x_a, x_b)
    assert r_a["stats"][:7] == r_b["stats"][:7]   # threshold / split-candidate statistics


CASES = [
    # (shape, dtype, alpha scale, opts, min fraction of iterations decided on the device).
    # At alpha0 = 2.5x the step every first trial of the large case is rejected, so the
    # speculative steady state (and with it device control) never starts: host control only.
    ((256, 16384, 32), np.float64, 1.0, {"maxit": 300}, 0.5),
    ((256, 16384, 32), np.float64, 2.5, {"maxit": 120}, 0.0),
    ((512, 1024, 16), np.float64, 1.0, {}, 0.5),
    ((512, 1024, 16), np.float64, 2.5, {}, 1e-4),   # rejections inside device-controlled runs
    ((512, 1024, 16), np.float32, 1.0, {}, 0.5),
    ((1024, 2048, 32), np.float64, 1.0, {"maxit": 400}, 0.5),
    # round 5: plans without the fused trial (C1's l = 2; n % 64 != 0) on the communicator
    # form of the speculative trial (A^T r, then k_prox_pgd from its slabs, dc_queue_comm)
    ((512, 1024, 2), np.float64, 1.0, {"maxit": 300}, 0.5),
    ((512, 1024, 2), np.float64, 2.5, {"maxit": 120}, 0.0),
    ((300, 1000, 4), np.float64, 1.0, {"maxit": 200}, 0.5),
]


@pytest.mark.parametrize("shape,dtype,scale,opts,frac", CASES)
def test_device_control_bit_identical(monkeypatch, shape, dtype, scale, opts, frac):
    host = _run(monkeypatch, 0, shape, dtype, scale, opts)
    dev = _run(monkeypatch, 8, shape, dtype, scale, opts)
    _same(dev, host)
    r_h, r_d = host[1], dev[1]
    assert r_h["stats"][7] == 0
    assert r_d["stats"][7] >= frac * r_d["k"], r_d["stats"]
    if frac >= 0.5:
        assert r_d["syncs"] < 0.1 * r_h["syncs"]


@pytest.mark.parametrize("window", [1, 3, 32])
def test_window_sizes(monkeypatch, window):
    shape, opts = (512, 1024, 16), {}
    _same(_run(monkeypatch, window, shape, opts=opts, alpha_scale=2.5),
          _run(monkeypatch, 0, shape, opts=opts, alpha_scale=2.5))


def test_run_in_slices(monkeypatch):
    shape = (512, 1024, 16)
    sliced = _run(monkeypatch, 8, shape, slices=7)
    whole = _run(monkeypatch, 0, shape)
    _same(sliced, whole)


def test_split_candidate_gather_form(monkeypatch):
    shape, opts = (256, 16384, 32), {"maxit": 150}
    env = {"GLX_SPLIT_CAND": "1"}
    _same(_run(monkeypatch, 8, shape, opts=opts, env=env, alpha_scale=1.5),
          _run(monkeypatch, 0, shape, opts=opts, env=env, alpha_scale=1.5))


def test_max_total_iters(monkeypatch):
    shape, opts = (512, 1024, 16), {"max_total_iters": 37}
    dev = _run(monkeypatch, 8, shape, opts=opts)
    assert dev[1]["k"] == 37
    _same(dev, _run(monkeypatch, 0, shape, opts=opts))


def test_oracle_parity_with_device_control(monkeypatch):
    """The default (device-controlled) run against the NumPy oracle: same k, objective to 1e-10."""
    from oracle import numpy_ref
    shape = (512, 1024, 16)
    A, b, x0, mu, alpha0 = _instance(*shape)
    x, r = _run(monkeypatch, 8, shape, alpha_scale=2.5)
    xr, kr, outr = numpy_ref.gl_ProxGD_primal(x0, A, b, mu, {"alpha0": alpha0 * 2.5})
    assert r["k"] == kr
    assert abs(r["fval"] - outr["fval"]) <= 1e-10 * abs(outr["fval"])
    assert r["stats"][7] > 0


# ---- FProxGD (solver.cpp fista_dc_run): the backtracking test (gl_FProxGD_primal.py:92-97), the
# next record and the stop rule on the device; split-candidate batches also check nnz(e_c)
# against the budget (code 3 ends the device batch, dense batches follow on the host path and
# are device-controlled again up to the A thr(x_k) restore).
FISTA_CASES = [
    ((512, 1024, 16), np.float64, 1.0, {}, {}, 0.5),
    ((512, 1024, 16), np.float64, 3.0, {}, {}, 0.3),      # backtracking rejections
    ((512, 1024, 16), np.float32, 1.0, {}, {}, 0.5),      # fp32 (C3's dtype)
    ((256, 16384, 32), np.float64, 1.0, {"maxit": 300}, {}, 0.5),
    ((256, 16384, 32), np.float64, 1.5, {"maxit": 200}, {"GLX_SPLIT_CAND": "1"}, 0.5),
    # a tight nnz budget: gathered batches trip it, dense runs and restores alternate
    ((256, 16384, 32), np.float64, 1.0, {"maxit": 400}, {"GLX_SPLIT_CAND": "1", "GLX_SPLIT_NNZ": "0.002"}, 0.3),
]


@pytest.mark.parametrize("shape,dtype,scale,opts,env,frac", FISTA_CASES)
def test_fista_device_control_bit_identical(monkeypatch, shape, dtype, scale, opts, env, frac):
    m = "gl_FProxGD_primal"
    host = _run(monkeypatch, 0, shape, dtype, scale, opts, env=env, method=m)
    dev = _run(monkeypatch, 8, shape, dtype, scale, opts, env=env, method=m)
    _same(dev, host)
    r_h, r_d = host[1], dev[1]
    assert r_h["stats"][7] == 0
    assert r_d["stats"][7] >= frac * r_d["k"], r_d["stats"]
    assert r_d["syncs"] < 0.5 * r_h["syncs"], (r_d["syncs"], r_h["syncs"])
    if env.get("GLX_SPLIT_NNZ"):
        assert r_d["stats"][3] > 0 and r_d["stats"][4] > 0 and r_d["stats"][6] > 1, r_d["stats"]


@pytest.mark.parametrize("window", [1, 3, 32])
def test_fista_window_sizes(monkeypatch, window):
    m, shape = "gl_FProxGD_primal", (512, 1024, 16)
    _same(_run(monkeypatch, window, shape, alpha_scale=3.0, method=m),
          _run(monkeypatch, 0, shape, alpha_scale=3.0, method=m))


def test_fista_run_in_slices_and_max_total(monkeypatch):
    m, shape = "gl_FProxGD_primal", (512, 1024, 16)
    _same(_run(monkeypatch, 8, shape, slices=7, method=m), _run(monkeypatch, 0, shape, method=m))
    dev = _run(monkeypatch, 8, shape, opts={"max_total_iters": 41}, method=m)
    assert dev[1]["k"] == 41
    _same(dev, _run(monkeypatch, 0, shape, opts={"max_total_iters": 41}, method=m))


def test_fista_oracle_parity_with_device_control(monkeypatch):
    from oracle import numpy_ref
    shape = (512, 1024, 16)
    A, b, x0, mu, alpha0 = _instance(*shape)
    x, r = _run(monkeypatch, 8, shape, alpha_scale=3.0, method="gl_FProxGD_primal")
    xr, kr, outr = numpy_ref.gl_FProxGD_primal(x0, A, b, mu, {"alpha0": alpha0 * 3.0})
    assert r["k"] == kr
    assert abs(r["fval"] - outr["fval"]) <= 1e-10 * abs(outr["fval"])
    assert r["stats"][7] > 0



@pytest.mark.parametrize("shape,scale", [((512, 1024, 2), 1.0), ((512, 1024, 2), 2.5), ((300, 1000, 4), 1.0),
                                         ((256, 512, 8), 1.0)])
def test_unfused_speculative_form_bit_identical(monkeypatch, shape, scale):
    """Round 5: with a plan that cannot fuse the trial into A^T r, host control runs the
    speculative trial as A^T r + k_prox_pgd from its slabs (GLX_UNFUSED_SPEC, default on): the
    same arithmetic in the same order as the separate gradient and trial (GLX_UNFUSED_SPEC=0)."""
    a = _run(monkeypatch, 0, shape, alpha_scale=scale, opts={"maxit": 200})
    b = _run(monkeypatch, 0, shape, alpha_scale=scale, opts={"maxit": 200}, env={"GLX_UNFUSED_SPEC": "0"})
    _same(a, b)
    assert a[1]["syncs"] <= b[1]["syncs"]
