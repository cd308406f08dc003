"""Multi-process (gloo, world_size 2 and 3) CPU tests of the row-sharded decomposition.

libglx's N-GPU path (src/comm.cpp, solver.cpp) keeps x replicated and row-shards A and b:
every rank forms r_g = A_g x - b_g, sums its squared norm and A_g^T r_g, and one sum
all-reduce produces the global sum of squares and gradient; all row-wise steps and all
branch decisions are then replicated. This test runs exactly that schedule with
torch.distributed (gloo) on top of the oracle's arithmetic and checks it reproduces the
unsharded oracle: same iteration count, objective within 1e-10, identical decisions on every
rank — the property the RCCL path relies on.
"""
import os
import socket
import warnings

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import numpy_ref as R


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _allreduce(arr):
    t = torch.from_numpy(np.ascontiguousarray(arr, dtype=np.float64))
    dist.all_reduce(t)
    return t.numpy()


def sharded_proxgd(x0, A_g, b_g, mu_0, opts):
    """ProxGD with the libglx N-GPU exchange pattern (one all-reduce per gradient and per
    squared-residual sum)."""
    o = {**R.PROXGD_DEFAULTS, **opts}
    thres, alpha0, coeff = o["thres"], o["alpha0"], o["line_search_attenuation_coeffi"]

    def half_sq(x):
        r = A_g @ x - b_g
        return 0.5 * float(_allreduce(np.array([np.sum(r ** 2)]))[0]), r

    hist = R._History(o["ftol"], use_sparsity=True)
    x = np.copy(x0)
    decisions = []
    for mu in (100 * mu_0, 10 * mu_0, mu_0):
        inner, stable = 0, 0
        while inner < o["maxit"]:
            g, _ = half_sq(x)
            hist.record(g + mu_0 * np.sum(R._group_norms(x)), R.sparsity(x))
            inner += 1
            stable = stable + 1 if hist.stable_step() else 0
            if stable > o["stable_len_threshold"]:
                break
            R._zero_small(x, thres)
            gx, r = half_sq(x)
            grad = _allreduce(A_g.T @ r)
            t = alpha0
            for i in range(o["maxit_line_search_iter"]):
                gt = (x - R._group_shrink(x - t * grad, t, mu, thres)) / t
                lhs, _ = half_sq(x - t * gt)
                ok = lhs <= gx - t * np.sum(grad * gt) + 0.5 * t * np.sum(gt ** 2)
                decisions.append(bool(ok))
                if ok:
                    break
                t *= coeff
            x = R._group_shrink(x - t * grad, t, mu, thres)
    g, _ = half_sq(x)
    return x, hist.k, g + mu_0 * np.sum(R._group_norms(x)), decisions


def _worker(rank, world, port, shape, seed, opts, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from glx.dist import shard_rows
        m, n, l = shape
        A, b, u, x0, mu = R.gen_data(m, n, l, seed)
        r0, r1 = shard_rows(m, world, rank)
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            x, k, fval, dec = sharded_proxgd(x0, A[r0:r1], b[r0:r1], mu, opts)
        q.put((rank, k, float(fval), dec, x))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_row_sharded_proxgd_matches_unsharded(world):
    shape, seed, opts = (96, 160, 4), 11, {"maxit": 40, "alpha0": R.step_size_for(96, 160)}
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, shape, seed, opts, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = sorted([q.get(timeout=240) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    A, b, u, x0, mu = R.gen_data(*shape, seed)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        xr, kr, outr = R.gl_ProxGD_primal(x0, A, b, mu, dict(opts))
    for rank, k, fval, dec, x in outs:
        assert k == kr
        assert abs(fval - float(outr["fval"])) <= 1e-10 * abs(float(outr["fval"]))
        np.testing.assert_allclose(x, xr, rtol=1e-8, atol=1e-12)
        assert dec == outs[0][3]                        # every rank took the same branches
        assert np.array_equal(x, outs[0][4])            # replicated state stays identical
