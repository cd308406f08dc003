"""Row-sharded solves with world size 2, 3 and 8 on ONE GPU (host-staged transport over gloo).

Every rank runs the full libglx N-GPU path of solver.cpp — local A_g x - b_g and A_g^T r_g, the
gradient and every squared-residual sum all-reduced, replicated row-wise steps and decisions —
with the all-reduces staged through host memory instead of RCCL (RCCL needs one GPU per rank).
ProxGD where n divides by the world size takes the row-sharded schedule instead (round 5,
iter_proxgd_shard): the gradient reduce-scattered, the trial on n / G rows, p's rows and the
partial sums all-gathered and combined in rank order (test_row_sharded_*).
Checks: every rank returns the same k, fval and bit-identical x; k equals the unsharded oracle's
and fval / f_hist agree to 1e-8 relative (fp64), as in tests/test_gpu_parity.py.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run_sharded(tmp_path, world, solver, m, n, l, dtype="f64", maxit=20, extra=(), threads=1,
                timeout=110):
    out = tmp_path / ("verdict_%s_%d.json" % (solver, world))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1",
           "--nproc-per-node", str(world), "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.join(ROOT, "tests", "dist_gpu_worker.py"),
           "--solver", solver, "--rows", str(m), "--cols", str(n), "--groups-l", str(l), "--dtype", dtype,
           "--maxit", str(maxit), "--out", str(out)] + list(extra)
    env = dict(os.environ, OMP_NUM_THREADS=str(threads))
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout)
    if p.returncode != 0:   # the first worker traceback, not just the launcher's summary
        i = p.stderr.find("Traceback")
        raise AssertionError(p.stderr[max(0, i):max(0, i) + 4000] + "\n...\n" + p.stderr[-1500:])
    with open(out) as fh:
        return json.load(fh)


@pytest.mark.parametrize("world,solver,shape", [
    (2, "gl_ProxGD_primal", (515, 1024, 16)),
    (3, "gl_ProxGD_primal", (515, 1024, 32)),
    (2, "gl_FProxGD_primal", (512, 1024, 32)),
    (3, "gl_SGD_primal", (1031, 256, 1)),
    (2, "gl_GD_primal", (512, 768, 4)),
])
def test_sharded_matches_oracle(tmp_path, world, solver, shape):
    v = run_sharded(tmp_path, world, solver, *shape)
    ranks = v["ranks"]
    assert len(ranks) == world
    for r in ranks[1:]:   # replicated decisions: identical results on every rank
        assert r["k"] == ranks[0]["k"] and r["fval"] == ranks[0]["fval"] and r["x_sha"] == ranks[0]["x_sha"]
    assert ranks[0]["k"] == v["oracle_k"]
    rel = abs(ranks[0]["fval"] - v["oracle_fval"]) / abs(v["oracle_fval"])
    assert rel < 1e-8, rel
    fh, fo = np.asarray(ranks[0]["f_hist"]), np.asarray(v["oracle_f_hist"])
    assert fh.shape == fo.shape
    assert np.max(np.abs(fh - fo) / np.abs(fo)) < 1e-8
    assert v["x_maxdiff"] <= 1e-6 * v["x_scale"]


@pytest.mark.parametrize("solver", ["gl_ProxGD_primal", "gl_FProxGD_primal"])
def test_sharded_split_candidate_forced(tmp_path, monkeypatch, solver):
    # the split-candidate trial (default only for A >= 768 MiB per rank) forced at a small shard,
    # on the all-reduce schedule (the row-sharded FProxGD runs the dense batch)
    monkeypatch.setenv("GLX_SPLIT_CAND", "1")
    v = run_sharded(tmp_path, 2, solver, 512, 1024, 32, maxit=25, extra=("--shard-rows", "2"))
    ranks = v["ranks"]
    assert ranks[0]["x_sha"] == ranks[1]["x_sha"] and ranks[0]["k"] == ranks[1]["k"]
    assert ranks[0]["k"] == v["oracle_k"]
    fh, fo = np.asarray(ranks[0]["f_hist"]), np.asarray(v["oracle_f_hist"])
    assert np.max(np.abs(fh - fo) / np.abs(fo)) < 1e-8
    assert v["x_maxdiff"] <= 1e-6 * v["x_scale"]


def test_sharded_proxgd_line_search_rejections(tmp_path):
    # alpha0 above 1/L: first trials are rejected and retried (k_prox_pgd), others accepted
    # (the trial staged into A @ [z | p_thr]); speculation is dropped and resumed around them
    v = run_sharded(tmp_path, 2, "gl_ProxGD_primal", 512, 1024, 32, maxit=25,
                    extra=("--alpha-scale", "2.5"))
    ranks = v["ranks"]
    assert ranks[0]["x_sha"] == ranks[1]["x_sha"] and ranks[0]["k"] == ranks[1]["k"]
    assert ranks[0]["k"] == v["oracle_k"]
    fh, fo = np.asarray(ranks[0]["f_hist"]), np.asarray(v["oracle_f_hist"])
    assert np.max(np.abs(fh - fo) / np.abs(fo)) < 1e-8
    assert v["x_maxdiff"] <= 1e-6 * v["x_scale"]


def test_sharded_fp32(tmp_path):
    v = run_sharded(tmp_path, 2, "gl_FProxGD_primal", 512, 1024, 16, dtype="f32", maxit=10)
    ranks = v["ranks"]
    assert ranks[0]["x_sha"] == ranks[1]["x_sha"]
    # fp32, 10 iterations per phase (not converged): measured 0.6e-6 .. 1.04e-6 relative on
    # different boxes. The fp32 oracle's own sgemm rounding depends on the host CPU's OpenBLAS
    # kernel, and one fp32 dot product over n = 1024 already carries ~sqrt(n) eps ~ 2e-6, so
    # the bar is 1e-5 here; the converged fp32 cases keep 1e-6 (test_gpu_parity.py).
    assert abs(ranks[0]["fval"] - v["oracle_fval"]) / abs(v["oracle_fval"]) < 1e-5


def test_sharded_continuous_subgradient(tmp_path):
    # alpha0 = 1 / max eig(sum_g A_g^T A_g): the Gram matrix is all-reduced across the shards
    v = run_sharded(tmp_path, 2, "gl_SGD_primal", 301, 256, 2, extra=["--csf"])
    ranks = v["ranks"]
    assert ranks[0]["x_sha"] == ranks[1]["x_sha"]
    assert ranks[0]["k"] == v["oracle_k"]
    assert abs(ranks[0]["fval"] - v["oracle_fval"]) / abs(v["oracle_fval"]) < 1e-8


def test_sharded_c5_shape_fprox_fp64(tmp_path):
    """C5's row-sharded FProxGD fp64 with C5's per-rank shard shape (16384 rows x 16384 x 32
    per rank, 4 GiB of A in all) at world size 2, two iterations per phase, against the
    unsharded oracle (gl_FProxGD_primal.py:110-151). The oracle uses 8 BLAS threads here."""
    v = run_sharded(tmp_path, 2, "gl_FProxGD_primal", 32768, 16384, 32, maxit=2, threads=8,
                    timeout=140)
    ranks = v["ranks"]
    assert ranks[0]["x_sha"] == ranks[1]["x_sha"] and ranks[0]["k"] == ranks[1]["k"]
    assert ranks[0]["k"] == v["oracle_k"] == 6
    rel = abs(ranks[0]["fval"] - v["oracle_fval"]) / abs(v["oracle_fval"])
    assert rel < 1e-8, rel
    fh, fo = np.asarray(ranks[0]["f_hist"]), np.asarray(v["oracle_f_hist"])
    assert np.max(np.abs(fh - fo) / np.abs(fo)) < 1e-8
    assert v["x_maxdiff"] <= 1e-6 * v["x_scale"]


@pytest.mark.timeout(400)
def test_sharded_c5_global_world8(tmp_path):
    """C5's global problem (131072 x 16384 x 32 fp64, 16 GiB of A; gl_FProxGD_primal.py:110-151
    row-sharded) split the 8-GPU way: 8 ranks of 16384 rows, one iteration per continuation
    phase, against the unsharded oracle on the same instance. The instance is ONE host copy in
    /dev/shm (each rank generates its own rows), so host RAM holds A once; all 8 ranks share the
    box's GPU through the host-staged transport."""
    v = run_sharded(tmp_path, 8, "gl_FProxGD_primal", 131072, 16384, 32, maxit=1, threads=16,
                    extra=("--shm",), timeout=380)
    ranks = v["ranks"]
    assert len(ranks) == 8
    for r in ranks[1:]:
        assert r["x_sha"] == ranks[0]["x_sha"] and r["k"] == ranks[0]["k"] and r["fval"] == ranks[0]["fval"]
    assert ranks[0]["k"] == v["oracle_k"] == 3
    rel = abs(ranks[0]["fval"] - v["oracle_fval"]) / abs(v["oracle_fval"])
    assert rel < 1e-8, rel
    fh, fo = np.asarray(ranks[0]["f_hist"]), np.asarray(v["oracle_f_hist"])
    assert fh.shape == fo.shape
    assert np.max(np.abs(fh - fo) / np.abs(fo)) < 1e-8
    assert v["x_maxdiff"] <= 1e-6 * v["x_scale"]


def _check_identical_and_oracle(v, world, bar=1e-8):
    ranks = v["ranks"]
    assert len(ranks) == world
    for r in ranks[1:]:   # every rank combines the same gathered sums: identical bits everywhere
        assert r["k"] == ranks[0]["k"] and r["fval"] == ranks[0]["fval"] and r["x_sha"] == ranks[0]["x_sha"]
        assert r["f_hist"] == ranks[0]["f_hist"]
    assert ranks[0]["k"] == v["oracle_k"]
    rel = abs(ranks[0]["fval"] - v["oracle_fval"]) / abs(v["oracle_fval"])
    assert rel < bar, rel
    fh, fo = np.asarray(ranks[0]["f_hist"]), np.asarray(v["oracle_f_hist"])
    assert fh.shape == fo.shape
    assert np.max(np.abs(fh - fo) / np.abs(fo)) < bar
    return ranks[0]


@pytest.mark.parametrize("world,shape,extra", [
    (2, (515, 1024, 16), ()),
    (3, (515, 1536, 32), ()),
    (8, (1024, 1024, 32), ()),
    (2, (512, 1024, 32), ("--alpha-scale", "2.5")),   # rejected first trials, retried on n/G rows
    (3, (600, 768, 5), ()),                           # l = 5: LPR 8 rows, no column bitmaps
])
def test_row_sharded_proxgd(tmp_path, world, shape, extra):
    """ProxGD's row-sharded schedule (reduce-scatter of A^T r, k_prox_pgd on n / G rows, one
    all-gather of p's rows and the partial sums, k_trial_split) against the unsharded oracle
    (gl_ProxGD_primal.py:73-132): k identical, f_hist within 1e-8, bit-identical on every rank."""
    v = run_sharded(tmp_path, world, "gl_ProxGD_primal", *shape, maxit=25,
                    extra=("--shard-rows", "1") + tuple(extra), timeout=150)
    r0 = _check_identical_and_oracle(v, world)
    assert ("rows=sharded x%d" % world) in r0["plan"], r0["plan"]
    assert v["x_maxdiff"] <= 1e-6 * v["x_scale"]


@pytest.mark.parametrize("extra_opts", [{"step_type": "fixed"}, {"exact_objective": 1}])
def test_row_sharded_other_modes(tmp_path, extra_opts):
    """The row-sharded schedule with the fixed step (every trial untested: the prologue's
    all-reduced sums each iteration) and with exact_objective (A p as a third right-hand side from
    the gathered p), world 2, against the unsharded oracle."""
    import json as _json
    v = run_sharded(tmp_path, 2, "gl_ProxGD_primal", 512, 1024, 32, maxit=25,
                    extra=("--shard-rows", "1", "--opts", _json.dumps(extra_opts)))
    r0 = _check_identical_and_oracle(v, 2)
    assert "rows=sharded x2" in r0["plan"]


@pytest.mark.parametrize("world,m,n,extra", [
    (2, 512, 1024, ()),
    (2, 512, 1024, ("--alpha-scale", "2.5")),
    (3, 1000, 1536, ()),   # ragged rows per rank (334 / 333 / 333), three ranks' chunk bitmaps
    (8, 1024, 1024, ()),   # 128 rows of x per rank: two bitmap words per rank and column
])
def test_row_sharded_split_candidate(tmp_path, monkeypatch, world, m, n, extra):
    """The split-candidate trial under the row-sharded schedule: p_thr, the masks and bitmaps of e
    are re-derived from the gathered p and the bitmap gather reads e from them. Round 6: in the
    speculative steady state the derive runs inside the next trial's dense pass (k_ax_lds DRV; its
    publisher workgroup combines the gathered sums) with A e as its extra workgroups (bitmaps from the
    all-gathered sums chunks), elsewhere in k_trial_split and k_at_gather_bm; GLX_SHARD_DERIVE=0
    (those two throughout) gives the same bits. alpha0 x 2.5: rejected first trials (the
    host-path trial, then the fused form again once speculation resumes)."""
    monkeypatch.setenv("GLX_SPLIT_CAND", "1")
    v = run_sharded(tmp_path, world, "gl_ProxGD_primal", m, n, 32, maxit=25,
                    extra=("--shard-rows", "1") + tuple(extra), timeout=150)
    r0 = _check_identical_and_oracle(v, world)
    assert "gather k_at_gather_bm" in r0["plan"] and ("rows=sharded x%d" % world) in r0["plan"], r0["plan"]
    assert "derive and A e in the dense pass" in r0["plan"], r0["plan"]
    monkeypatch.setenv("GLX_SHARD_DERIVE", "0")
    w = run_sharded(tmp_path, world, "gl_ProxGD_primal", m, n, 32, maxit=25,
                    extra=("--shard-rows", "1") + tuple(extra), timeout=150)
    w0 = w["ranks"][0]
    assert "k_trial_split" in w0["plan"], w0["plan"]
    assert w0["k"] == r0["k"] and w0["x_sha"] == r0["x_sha"] and w0["f_hist"] == r0["f_hist"]


def test_row_sharded_matches_allreduce_schedule(tmp_path):
    """Both multi-GPU schedules on the same instance: same k, f_hist within 1e-12 of each other
    (they differ only in the order the trial sums are added)."""
    a = run_sharded(tmp_path, 2, "gl_ProxGD_primal", 515, 1024, 32, maxit=25, extra=("--shard-rows", "1"))
    b = run_sharded(tmp_path, 2, "gl_ProxGD_primal", 515, 1024, 32, maxit=25, extra=("--shard-rows", "2"))
    ra, rb = a["ranks"][0], b["ranks"][0]
    assert "rows=sharded" in ra["plan"] and "rows=sharded" not in rb["plan"]
    assert ra["k"] == rb["k"]
    fa, fb = np.asarray(ra["f_hist"]), np.asarray(rb["f_hist"])
    assert np.max(np.abs(fa - fb) / np.abs(fb)) < 1e-12


def test_row_sharded_fp32(tmp_path):
    """fp32 ProxGD (the dense [z | p_thr] batch: k_trial_split re-derives z = x - t G_t)."""
    v = run_sharded(tmp_path, 2, "gl_ProxGD_primal", 512, 1024, 16, dtype="f32", maxit=10,
                    extra=("--shard-rows", "1"))
    ranks = v["ranks"]
    assert ranks[0]["x_sha"] == ranks[1]["x_sha"] and "rows=sharded" in ranks[0]["plan"]
    assert abs(ranks[0]["fval"] - v["oracle_fval"]) / abs(v["oracle_fval"]) < 1e-5   # as test_sharded_fp32


@pytest.mark.parametrize("world", [2, 3])
def test_host_reduce_scatter_all_gather(tmp_path, world):
    """The row-sharded schedule's collectives on the host transport: reduce-scatter sums match
    NumPy, the all-gather is bit-exact (-0.0, NaN, -inf chunks included)."""
    v = run_sharded(tmp_path, world, "collectives", 1, 1, 1)
    assert v["ok"] == [True] * world


def test_row_sharded_needs_divisible_rows(tmp_path):
    """shard_rows = 1 with n % G != 0 is refused; auto (0) keeps the all-reduce schedule."""
    v = run_sharded(tmp_path, 3, "gl_ProxGD_primal", 515, 1024, 16, maxit=5, extra=("--shard-rows", "0"))
    assert "rows=sharded" not in v["ranks"][0]["plan"]
    with pytest.raises(AssertionError, match="n % ranks == 0"):
        run_sharded(tmp_path, 3, "gl_ProxGD_primal", 515, 1024, 16, maxit=5, extra=("--shard-rows", "1"))


@pytest.mark.timeout(600)
def test_row_sharded_ns_world8_whole_solve(tmp_path):
    """the exact path the driver's 8-GPU strong-scaling run takes
    (bench.py --gpus 8: gl_ProxGD_primal fp64 at (8192, 16384, 32), 1024 rows of A per rank,
    default options: the row-sharded schedule, the split-candidate trial with the bitmap gather,
    a 4 MiB reduce-scatter and all-gather per iteration) as 8 host-staged ranks sharing the box's
    GPU, a whole solve from x0 against the reference's own run of the same call
    (tests/golden/ns_gl_ProxGD_primal.npz, gl_ProxGD_primal.py:9-146): k = 2680, fval and every
    f_hist entry within 1e-8, x within 1e-6 of max|x|, bit-identical on all 8 ranks, and the plan
    names the row-sharded schedule and the bitmap gather."""
    v = run_sharded(tmp_path, 8, "gl_ProxGD_primal", 8192, 16384, 32, threads=2,
                    extra=("--ns-golden", "ns_gl_ProxGD_primal"), timeout=580)
    r0 = _check_identical_and_oracle(v, 8)
    assert r0["k"] == 2680
    assert "rows=sharded x8" in r0["plan"] and "gather k_at_gather_bm" in r0["plan"], r0["plan"]
    assert "derive and A e in the dense pass" in r0["plan"], r0["plan"]
    assert v["x_maxdiff"] <= 1e-6 * v["x_scale"]


def test_stalled_rank_watchdog_host_transport(tmp_path):
    """one rank of a row-sharded ProxGD solve stops answering collectives
    (its host transport callback never returns after 10 calls); the other ranks block inside the
    collective. Every rank's glx.watchdog (armed as bench.py arms it for N > 1) prints its
    diagnostic — rank, phase, the session's progress record (iterations, collectives issued) and
    the communicator's (collectives issued / completed) — and the ranks leave with exit code 3,
    within the deadline instead of at an outer time limit."""
    import time
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "dist_gpu_worker.py"), "--solver", "gl_ProxGD_primal",
           "--rows", "512", "--cols", "1024", "--groups-l", "32", "--maxit", "200",
           "--out", str(tmp_path / "unused.json"),
           "--stall-rank", "1", "--stall-after", "10", "--watchdog-s", "20"]
    t0 = time.monotonic()
    p = subprocess.run(cmd, env=dict(os.environ, OMP_NUM_THREADS="1"), capture_output=True, text=True,
                       timeout=110)
    elapsed = time.monotonic() - t0
    msg = p.stderr
    assert p.returncode != 0
    assert elapsed < 100, elapsed
    assert "glx watchdog: rank 0 of 2: dist_gpu_worker stall check passed its deadline of 20 s" in msg, msg[-3000:]
    assert "session: {'k':" in msg and "'collectives_issued':" in msg, msg[-3000:]
    assert "communicator: {'issued':" in msg, msg[-3000:]


@pytest.mark.parametrize("world,shape,extra", [
    (2, (515, 1024, 16), ()),
    (3, (515, 1536, 32), ()),
    (8, (1024, 1024, 32), ()),
    (2, (512, 1024, 32), ("--alpha-scale", "3.0")),   # backtracking: rejected trials on n/G rows
    (3, (600, 768, 5), ()),
])
def test_row_sharded_fprox(tmp_path, world, shape, extra):
    """Round 6: FProxGD's row-sharded schedule (reduce-scatter of A^T r,
    k_fista_trial on n / G rows, one all-gather of xc's rows and the partial sums, k_fista_split
    re-deriving v_next and y_next on every rank) against the unsharded oracle
    (gl_FProxGD_primal.py:89-103, 136-147): k identical, f_hist within 1e-8, bit-identical on
    every rank."""
    v = run_sharded(tmp_path, world, "gl_FProxGD_primal", *shape, maxit=25,
                    extra=("--shard-rows", "1") + tuple(extra), timeout=150)
    r0 = _check_identical_and_oracle(v, world)
    assert ("rows=sharded x%d" % world) in r0["plan"] and "k_fista_split" in r0["plan"], r0["plan"]
    assert v["x_maxdiff"] <= 1e-6 * v["x_scale"]


def test_row_sharded_fprox_matches_allreduce_schedule(tmp_path):
    """Both FProxGD multi-GPU schedules on one instance: the all-reduce schedule with device
    control and the row-sharded one agree (same k, f_hist within 1e-12: they differ only in the
    order the trial sums are added)."""
    a = run_sharded(tmp_path, 2, "gl_FProxGD_primal", 515, 1024, 32, maxit=25, extra=("--shard-rows", "1"))
    b = run_sharded(tmp_path, 2, "gl_FProxGD_primal", 515, 1024, 32, maxit=25, extra=("--shard-rows", "2"))
    ra, rb = a["ranks"][0], b["ranks"][0]
    assert "rows=sharded" in ra["plan"] and "rows=sharded" not in rb["plan"]
    assert ra["k"] == rb["k"]
    fa, fb = np.asarray(ra["f_hist"]), np.asarray(rb["f_hist"])
    assert np.max(np.abs(fa - fb) / np.abs(fb)) < 1e-12


def test_row_sharded_fprox_c5_shard_shape(tmp_path):
    """C5's per-rank shard (16384 rows x 16384 x 32 fp64) on the row-sharded FProxGD schedule
    (forced: auto keeps the all-reduce schedule with device control for 2 GiB shards), world 2,
    two iterations per phase, against the unsharded oracle."""
    v = run_sharded(tmp_path, 2, "gl_FProxGD_primal", 32768, 16384, 32, maxit=2, threads=8,
                    extra=("--shard-rows", "1"), timeout=140)
    r0 = _check_identical_and_oracle(v, 2)
    assert r0["k"] == 6 and "k_fista_split" in r0["plan"]
    assert v["x_maxdiff"] <= 1e-6 * v["x_scale"]
