"""Multi-process (gloo, world_size 2 and 3) CPU tests of the row-sharded decomposition.

Two schedules: the gradient all-reduce (below) and, round 5, the row-sharded trial
(sharded_proxgd_rows: reduce-scatter, the trial on n / world rows, all-gather of p and of the
partial sums in rank order), the schedule libglx's iter_proxgd_shard runs on the GPUs.

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


def _gather_rows(rows, world):
    """all-gather of equal row blocks in rank order (the row-sharded schedule's p exchange)"""
    t = torch.from_numpy(np.ascontiguousarray(rows, dtype=np.float64))
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    return np.concatenate([q.numpy() for q in parts], axis=0)


def _gather_sum(vals, world):
    """every rank's partial sums, all-gathered and added in rank order (k_shard_combine)"""
    t = torch.from_numpy(np.asarray(vals, dtype=np.float64))
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    acc = parts[0].numpy().copy()
    for q in parts[1:]:
        acc = acc + q.numpy()
    return acc


def sharded_proxgd_rows(x0, A_g, b_g, mu_0, opts, rank, world):
    """ProxGD with the round-5 row-sharded exchange (solver.cpp iter_proxgd_shard): the gradient
    reduce-scattered (this rank keeps its n / world rows), the trial's prox and sums on those rows
    only, p's rows and the partial sums all-gathered and added in rank order; z follows from x and
    the gathered p (k_trial_split)."""
    o = {**R.PROXGD_DEFAULTS, **opts}
    thres, alpha0, coeff = o["thres"], o["alpha0"], o["line_search_attenuation_coeffi"]
    n = x0.shape[0]
    rows = n // world
    own = slice(rank * rows, (rank + 1) * rows)

    def half_sq(x):
        r = A_g @ x - b_g
        return 0.5 * float(_gather_sum([np.sum(r ** 2)], world)[0]), r

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
            g_own = _allreduce(A_g.T @ r)[own]          # reduce-scatter: this rank's rows
            t = alpha0
            for i in range(o["maxit_line_search_iter"]):
                p_own = R._group_shrink(x[own] - t * g_own, t, mu, thres)
                gt_own = (x[own] - p_own) / t
                sums = _gather_sum([np.sum(g_own * gt_own), np.sum(gt_own ** 2)], world)
                p = _gather_rows(p_own, world)
                z = x - t * ((x - p) / t)
                lhs, _ = half_sq(z)
                ok = lhs <= gx - t * sums[0] + 0.5 * t * sums[1]
                decisions.append(bool(ok))
                if ok:
                    break
                t *= coeff
            x = _gather_rows(R._group_shrink(x[own] - t * g_own, t, mu, thres), world)
    g, _ = half_sq(x)
    return x, hist.k, g + mu_0 * np.sum(R._group_norms(x)), decisions


def _worker(rank, world, port, shape, seed, opts, q, schedule="allreduce"):
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
            if schedule == "rows":
                x, k, fval, dec = sharded_proxgd_rows(x0, A[r0:r1], b[r0:r1], mu, opts, rank, world)
            else:
                x, k, fval, dec = sharded_proxgd(x0, A[r0:r1], b[r0:r1], mu, opts)
        q.put((rank, k, float(fval), dec, x))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,schedule", [(2, "allreduce"), (3, "allreduce"), (2, "rows"), (3, "rows")])
def test_row_sharded_proxgd_matches_unsharded(world, schedule):
    shape, seed, opts = (96, 168, 4), 11, {"maxit": 40, "alpha0": R.step_size_for(96, 168)}
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, shape, seed, opts, q, schedule))
             for r in range(world)]
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
