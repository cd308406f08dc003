"""The RCCL path of libglx on one GPU (world size 1).

With a communicator, the solver sums the A^T r slabs, all-reduces the gradient and every
squared-residual sum over RCCL, and feeds S = 1 arrays to the row kernels — the exact code path
every rank runs at N GPUs. With one rank the all-reduce is an identity, so the result must be
bit-identical to the communicator-free run (which sums the slabs inside the prox kernel, in the
same slab order; GLX_ATR_FUSE_SPLIT=0 keeps that run off the fused A^T R + trial kernel, whose
trial sums are added in another order). N > 1 is covered by tests/test_dist_cpu.py (gloo) and the driver's 8-GPU run.
"""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def comm():
    import torch.distributed as dist
    from glx.dist import Comm
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("gloo", rank=0, world_size=1)
    c = Comm.from_torch_distributed()
    yield c
    c.close()
    dist.destroy_process_group()


def test_allreduce_identity_world1(comm):
    t = torch.arange(1000, dtype=torch.float64, device="cuda")
    ref = t.clone()
    comm.allreduce_(t)
    torch.cuda.synchronize()
    assert torch.equal(t, ref)


def test_reduce_scatter_all_gather_world1(comm):
    """RCCL reduce-scatter / all-gather at world size 1 (the row-sharded schedule's collectives):
    identities."""
    for dt in (torch.float64, torch.float32):
        t = torch.randn(4096, dtype=dt, device="cuda")
        ref = t.clone()
        comm.reduce_scatter_(t)
        comm.all_gather_(t)
        torch.cuda.synchronize()
        assert torch.equal(t, ref)


def test_shard_timing_model_world1(comm, monkeypatch):
    """opts shard_model=8 at world size 1 (bench.py --shard-model 8 --force-comm): the per-rank
    schedule of 8 ranks — the trial on n / 8 rows — runs and says so; its iterates are not a
    solve, so glx.solve and the C ABI's glx_solve refuse it, and the environment variable of
    round 5 no longer turns it on."""
    import glx
    from oracle import numpy_ref
    A, b, u, x0, mu = numpy_ref.gen_data(256, 1024, 32, 7)
    At, bt, xt = (torch.from_numpy(a).to("cuda", torch.float64) for a in (A, b, x0))
    opts = {"alpha0": numpy_ref.step_size_for(256, 1024), "maxit": 10}
    s = glx.Session("gl_ProxGD_primal", xt.clone(), At, bt, mu, dict(opts, shard_model=8), comm=comm)
    assert "rows=sharded x8 (timing model)" in s.describe()
    done = s.run(12)
    s.close()
    assert done == 12
    with pytest.raises(ValueError, match="timing model"):
        glx.solve("gl_ProxGD_primal", xt.clone(), At, bt, mu, dict(opts, shard_model=8), comm=comm)
    monkeypatch.setenv("GLX_SHARD_MODEL", "8")
    s = glx.Session("gl_ProxGD_primal", xt.clone(), At, bt, mu, opts, comm=comm)
    assert "timing model" not in s.describe()
    s.close()


@pytest.mark.parametrize("solver,shape,dtype", [
    ("gl_ProxGD_primal", (512, 1024, 32), torch.float64),
    ("gl_FProxGD_primal", (512, 1024, 16), torch.float64),
    ("gl_SGD_primal", (1024, 256, 1), torch.float64),
    ("gl_FProxGD_primal", (512, 1024, 32), torch.float32),
])
def test_comm_path_bit_identical_world1(comm, monkeypatch, solver, shape, dtype):
    import glx
    monkeypatch.setenv("GLX_ATR_FUSE_SPLIT", "0")
    from oracle import numpy_ref
    m, n, l = shape
    A, b, u, x0, mu = numpy_ref.gen_data(m, n, l, 7)
    At, bt, xt = (torch.from_numpy(a).to("cuda", dtype) for a in (A, b, x0))
    opts = {"alpha0": numpy_ref.step_size_for(m, n), "maxit": 15}
    outs = []
    for c in (None, comm):
        x = xt.clone()
        s = glx.Session(solver, x, At, bt, mu, opts, comm=c)
        s.run(0)
        res = s.finish()
        s.close()
        torch.cuda.synchronize()
        outs.append((x.cpu().numpy(), res))
    (x0_, r0), (x1_, r1) = outs
    assert r0["k"] == r1["k"]
    assert np.array_equal(np.asarray(r0["f_hist"]), np.asarray(r1["f_hist"]))
    assert np.array_equal(x0_, x1_)
