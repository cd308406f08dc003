"""Sampled HIP-event kernel timing (opts profile = k: every k-th A@x / A^T r launch).

bench.py derives the roofline's average launch time from these events, so the count of timed
launches must follow the sampling rule and the times must be positive and per-launch sane.
"""
import math

import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("every", [0, 1, 4])
def test_sampled_kernel_timing(every):
    import glx
    from oracle import numpy_ref
    m, n, l = 512, 2048, 32
    A, b, _, x0, mu = numpy_ref.gen_data(m, n, l, 7)
    At, bt, xt = (torch.from_numpy(a).cuda() for a in (A, b, x0))
    opts = {"alpha0": numpy_ref.step_size_for(m, n), "maxit": 60, "profile": every}
    s = glx.Session("gl_ProxGD_primal", xt, At, bt, mu, opts)
    s.run(30)
    (ax_n, ax_ms), (atr_n, atr_ms) = s.kernel_time(0), s.kernel_time(1)
    res = s.finish()
    s.close()
    if every == 0:
        assert ax_n == 0 and atr_n == 0
        return
    # launches made before kernel_time() was read: all but the finish() epilogue's
    assert 0 < ax_n <= math.ceil(res["ax_calls"] / every)
    assert ax_n >= (res["ax_calls"] - 4) // every
    assert 0 < atr_n <= math.ceil(res["atr_calls"] / every)
    assert 0 < ax_ms / ax_n < 50 and 0 < atr_ms / atr_n < 50   # ms per launch at this size
