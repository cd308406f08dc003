"""One rank of the row-sharded GPU solve (launched by tests/test_gpu_dist.py via
torch.distributed.run). All ranks share cuda:0 and talk through libglx's host-staged transport
(glx_comm_create_host over gloo) — the same solver code path every rank runs over RCCL on an
8-GPU node, minus the transport. ``--transport rccl`` uses RCCL instead (needs one GPU per rank).

Rank g solves rows [g*m/N, (g+1)*m/N) of the instance; rank 0 also runs the unsharded CPU oracle
(test infrastructure) and writes a JSON verdict with every rank's k, fval and x digest.
"""
import argparse
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "convex-optimization_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--solver", default="gl_ProxGD_primal")
    ap.add_argument("--rows", dest="m", type=int, default=515)
    ap.add_argument("--cols", dest="n", type=int, default=1024)
    ap.add_argument("--groups-l", dest="l", type=int, default=16)
    ap.add_argument("--dtype", default="f64")
    ap.add_argument("--maxit", type=int, default=20)
    ap.add_argument("--transport", default="host", choices=["host", "rccl"])
    ap.add_argument("--csf", action="store_true", help="continuous_subgradient_flag (SGD/GD)")
    ap.add_argument("--alpha-scale", type=float, default=1.0,
                    help="alpha0 = scale / (sqrt(m) + sqrt(n))^2 (> 1: line-search rejections)")
    ap.add_argument("--shm", action="store_true",
                    help="one host copy of the instance in /dev/shm, each rank generating its own rows")
    ap.add_argument("--shard-rows", type=int, default=None,
                    help="opts shard_rows (ProxGD: 0 auto, 1 the row-sharded step, 2 all-reduce)")
    ap.add_argument("--opts", default="{}", help="more solver options (JSON)")
    ap.add_argument("--stall-rank", type=int, default=-1,
                    help="this rank's host all-reduce callback never returns after --stall-after "
                         "calls (the other ranks block in the collective); with --watchdog-s")
    ap.add_argument("--stall-after", type=int, default=10)
    ap.add_argument("--watchdog-s", type=float, default=0.0)
    ap.add_argument("--ns-golden", default=None,
                    help="solve the reference's own instance of tests/golden/<stem>.npz (main.py "
                         "gen_data, b = the reference run's A u) with its opts, checked against that "
                         "run instead of the oracle")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()

    import glx
    from glx.dist import Comm, shard_rows
    from oracle import numpy_ref

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = 0 if a.transport == "host" else int(os.environ.get("GLX_TEST_DEVICE", os.environ.get("LOCAL_RANK", "0")))
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    comm = Comm.host_staged() if a.transport == "host" else Comm.from_torch_distributed()

    if a.solver == "collectives":
        collectives_check(comm, rank, world, a.out)
        comm.close()
        dist.destroy_process_group()
        return
    if a.stall_rank >= 0:
        stall_check(a, comm, rank, world)   # exits through the watchdog
        return
    if a.ns_golden is not None:
        ns_golden(a, comm, rank, world)
        comm.close()
        dist.destroy_process_group()
        return
    r0, r1 = shard_rows(a.m, world, rank)
    shm_path = None
    if a.shm:
        shm_path = "/dev/shm/glx_dist_%d_%s" % (world, os.environ.get("MASTER_PORT", "0"))
        A, b, x0, mu = shm_instance(shm_path, a.m, a.n, a.l, 11, rank, r0, r1)
    else:
        A, b, u, x0, mu = numpy_ref.gen_data(a.m, a.n, a.l, 11)
    if a.dtype == "f32":
        A, b, x0 = (v.astype(np.float32) for v in (A, b, x0))
    opts = {"alpha0": a.alpha_scale * numpy_ref.step_size_for(a.m, a.n), "maxit": a.maxit}
    if a.csf:
        opts["continuous_subgradient_flag"] = True
    if a.shard_rows is not None:
        opts["shard_rows"] = a.shard_rows
    opts.update(json.loads(a.opts))
    x, k, out = glx.solve(a.solver, x0, A[r0:r1], b[r0:r1], mu, dict(opts), comm=comm)
    digest = hashlib.sha256(np.ascontiguousarray(x).tobytes()).hexdigest()
    mine = {"rank": rank, "k": int(k), "fval": float(out["fval"]), "x_sha": digest,
            "f_hist": [float(v) for v in out["f_hist"]], "plan": out["glx"]["plan"]}
    gathered = [None] * world
    dist.all_gather_object(gathered, mine)
    if rank == 0:
        xr, kr, outr = numpy_ref.SOLVERS[a.solver](x0, A, b, mu, dict(opts))
        verdict = {"ranks": gathered, "oracle_k": int(kr), "oracle_fval": float(outr["fval"]),
                   "oracle_f_hist": [float(v) for v in outr["f_hist"]],
                   "x_maxdiff": float(np.max(np.abs(x.astype(np.float64) - xr.astype(np.float64)))),
                   "x_scale": float(np.max(np.abs(xr)))}
        with open(a.out, "w") as fh:
            json.dump(verdict, fh)
    comm.close()
    if shm_path is not None:
        dist.barrier()
        if rank == 0:
            os.unlink(shm_path)
    dist.destroy_process_group()


def stall_check(a, comm, rank, world):
    """A row-sharded ProxGD solve whose rank a.stall_rank stops answering collectives: its host
    transport's callback (torch.distributed.all_reduce over gloo) sleeps instead of joining after
    a.stall_after calls. Every rank arms glx.watchdog with the session's and the communicator's
    progress records as probes (as bench.py does for N > 1); the test expects every rank to
    leave with the watchdog's exit code and diagnostic well before any outer limit."""
    import time
    import glx
    from glx.watchdog import Watchdog
    from oracle import numpy_ref
    # the stalled rank's own deadline is later, so the blocked ranks' diagnostics are the ones
    # the launcher sees first (it tears the others down after the first exit)
    dl = a.watchdog_s * (3 if rank == a.stall_rank else 1)
    wd = Watchdog(dl, "dist_gpu_worker stall check", rank=rank, world=world).start()
    wd.probe("communicator", comm.progress)
    calls = [0]
    orig = dist.all_reduce

    def all_reduce(t, *args, **kw):
        calls[0] += 1
        if rank == a.stall_rank and calls[0] > a.stall_after:
            time.sleep(3600)
        return orig(t, *args, **kw)
    dist.all_reduce = all_reduce   # the host transport's callback looks it up at call time
    from glx.dist import shard_rows
    A, b, u, x0, mu = numpy_ref.gen_data(a.m, a.n, a.l, 11)
    r0, r1 = shard_rows(a.m, world, rank)
    opts = {"alpha0": numpy_ref.step_size_for(a.m, a.n), "maxit": a.maxit}
    x = torch.from_numpy(x0).cuda()
    s = glx.Session(a.solver, x, torch.from_numpy(np.ascontiguousarray(A[r0:r1])).cuda(),
                    torch.from_numpy(np.ascontiguousarray(b[r0:r1])).cuda(), mu, opts, comm=comm)
    wd.probe("session", s.progress)
    wd.phase = "solve"
    s.run(0)
    raise SystemExit("the stalled solve returned (the watchdog should have ended this rank)")


def ns_golden(a, comm, rank, world):
    """The exact path of the driver's 8-GPU strong-scaling run (bench.py --gpus N): the reference's
    gen_data instance at the north-star size (main.py:37-51; b from the reference's own run,
    tests/golden/ns_instance_b.npz), the reference run's opts, every other option at its default
    (shard_rows auto, the split-candidate gate), a whole solve. Every rank reports k, fval, its
    f_hist, the digest of x and the plan; rank 0 adds the reference run's k / fval / f_hist."""
    import glx
    from oracle import numpy_ref
    gold_dir = os.path.join(ROOT, "tests", "golden")
    meta = json.load(open(os.path.join(gold_dir, a.ns_golden + ".json")))
    m, n, l = meta["m"], meta["n"], meta["l"]
    A, _, u, x0, mu = numpy_ref.gen_data(m, n, l, meta["seed"])
    b = np.load(os.path.join(gold_dir, "ns_instance_b.npz"))["b"]
    sha = lambda v: hashlib.sha256(np.ascontiguousarray(v).tobytes()).hexdigest()
    assert sha(A) == meta["sha256"]["A"] and sha(x0) == meta["sha256"]["x0"] and sha(b) == meta["sha256"]["b"]
    from glx.dist import shard_rows
    r0, r1 = shard_rows(m, world, rank)
    Ad = torch.from_numpy(np.ascontiguousarray(A[r0:r1])).cuda()
    del A
    bd = torch.from_numpy(np.ascontiguousarray(b[r0:r1])).cuda()
    x, k, out = glx.solve(a.solver, torch.from_numpy(x0).cuda(), Ad, bd, mu, dict(meta["opts"]), comm=comm)
    torch.cuda.synchronize()
    xh = x.cpu().numpy()
    mine = {"rank": rank, "k": int(k), "fval": float(out["fval"]), "x_sha": sha(xh),
            "f_hist": [float(v) for v in out["f_hist"]], "plan": out["glx"]["plan"],
            "tt": float(out["tt"])}
    gathered = [None] * world
    dist.all_gather_object(gathered, mine)
    if rank == 0:
        gold = np.load(os.path.join(gold_dir, a.ns_golden + ".npz"))
        xr = gold["x"].astype(np.float64)
        verdict = {"ranks": gathered, "oracle_k": int(gold["k"]), "oracle_fval": float(gold["fval"]),
                   "oracle_f_hist": [float(v) for v in gold["f_hist"]],
                   "x_maxdiff": float(np.max(np.abs(xh - xr))), "x_scale": float(np.max(np.abs(xr))),
                   "oracle": "the reference's own run (tests/golden/%s.npz)" % a.ns_golden}
        with open(a.out, "w") as fh:
            json.dump(verdict, fh)


def collectives_check(comm, rank, world, out):
    """glx_comm_reduce_scatter / glx_comm_all_gather on the host transport: chunk sums against
    NumPy and a bit-exact gather (signed zeros, NaN and infinities included)."""
    ok = True
    for dt, npdt in ((torch.float64, np.float64), (torch.float32, np.float32)):
        chunk = 1000
        full = [np.random.default_rng(100 + r).standard_normal(world * chunk).astype(npdt) for r in range(world)]
        t = torch.from_numpy(full[rank].copy()).cuda()
        comm.reduce_scatter_(t)
        torch.cuda.synchronize()
        want = full[0][rank * chunk:(rank + 1) * chunk].astype(np.float64)
        for r in range(1, world):
            want = want + full[r][rank * chunk:(rank + 1) * chunk]
        got = t.cpu().numpy()[rank * chunk:(rank + 1) * chunk].astype(np.float64)
        ok &= bool(np.allclose(got, want, rtol=1e-5 if npdt == np.float32 else 1e-13, atol=1e-6))
        src = [np.random.default_rng(200 + r).standard_normal(chunk).astype(npdt) for r in range(world)]
        for r in range(world):
            src[r][:4] = np.array([-0.0, 0.0, np.nan, -np.inf], dtype=npdt)
        t = torch.full((world * chunk,), 7.0, dtype=dt, device="cuda")
        t[rank * chunk:(rank + 1) * chunk] = torch.from_numpy(src[rank]).cuda()
        comm.all_gather_(t)
        torch.cuda.synchronize()
        ok &= t.cpu().numpy().tobytes() == np.concatenate(src).tobytes()
    import torch.distributed as dist
    res = [None] * world
    dist.all_gather_object(res, ok)
    if rank == 0:
        with open(out, "w") as fh:
            json.dump({"ok": res}, fh)


def shm_instance(path, m, n, l, seed, rank, r0, r1):
    """The instance as ONE host copy in shared memory (C5's global problem is 16 GiB of A): rank
    0 creates the file, every rank fills its own rows of A from a per-shard seed (seed + rank,
    SURVEY §8d's C5 recipe) and its rows of b = A u; u (10 % row-sparse) and x0 come from the
    common seed, drawn in gen_data's order (main.py:41-47). Returns memory-mapped views."""
    import torch.distributed as dist
    nbytes = 8 * (m * n + m * l)
    if rank == 0:
        with open(path, "wb") as fh:
            fh.truncate(nbytes)
    dist.barrier()
    mm = np.memmap(path, dtype=np.float64, mode="r+", shape=(m * n + m * l,))
    A = mm[:m * n].reshape(m, n)
    b = mm[m * n:].reshape(m, l)
    gen = np.random.Generator(np.random.MT19937(seed=seed))
    k = round(n * 0.1)
    support = gen.permutation(n)[:k]
    u = np.zeros(shape=(n, l))
    u[support, :] = gen.standard_normal(size=(k, l))
    x0 = gen.standard_normal(size=(n, l))
    rows = np.random.Generator(np.random.MT19937(seed=seed * 1000 + 1 + rank))
    for c0 in range(r0, r1, 1024):
        c1 = min(r1, c0 + 1024)
        rows.standard_normal(out=A[c0:c1])
        b[c0:c1] = A[c0:c1] @ u
    mm.flush()
    dist.barrier()
    return A, b, x0, 1e-2


if __name__ == "__main__":
    main()
