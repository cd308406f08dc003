"""One rank of a row-sharded device-control twin (launched by tests/test_gpu_dc_dist.py through
torch.distributed.run). All ranks share cuda:0 and exchange through libglx's host-staged
transport. For each GLX_DC_BATCH window in --windows the rank runs the same session (host
control for window 0), and rank 0 writes every rank's k, f_hist, fval, iterate digest, stats and
syncs to --out.
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
    ap.add_argument("--shape", required=True)            # m,n,l
    ap.add_argument("--dtype", default="f64")
    ap.add_argument("--alpha-scale", type=float, default=1.0)
    ap.add_argument("--opts", default="{}")
    ap.add_argument("--env", default="{}")
    ap.add_argument("--windows", default="0,8")
    ap.add_argument("--slices", type=int, default=0)
    ap.add_argument("--out", required=True)
    ap.add_argument("--method", default="gl_ProxGD_primal")
    ap.add_argument("--mu", type=float, default=None, help="mu0 (default: gen_data's)")
    a = ap.parse_args()

    import glx
    from glx.dist import Comm, shard_rows
    from oracle import numpy_ref

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    comm = Comm.host_staged()
    for k, v in json.loads(a.env).items():
        os.environ[k] = v
    m, n, l = (int(v) for v in a.shape.split(","))
    A, b, u, x0, mu = numpy_ref.gen_data(m, n, l, 2024)
    if a.mu is not None:
        mu = a.mu
    dt = np.float64 if a.dtype == "f64" else np.float32
    r0, r1 = shard_rows(m, world, rank)
    opts = {"alpha0": a.alpha_scale * numpy_ref.step_size_for(m, n)}
    opts.update(json.loads(a.opts))
    runs = {}
    for w in (int(v) for v in a.windows.split(",")):
        os.environ["GLX_DC_BATCH"] = str(w)
        At, bt, xt = (torch.from_numpy(np.ascontiguousarray(v.astype(dt))).cuda()
                      for v in (A[r0:r1], b[r0:r1], x0))
        s = glx.Session(a.method, xt, At, bt, mu, dict(opts), comm=comm)
        if a.slices:
            while not s.finished:
                s.run(a.slices)
        else:
            s.run(0)
        res = s.finish()
        s.close()
        torch.cuda.synchronize()
        x = xt.cpu().numpy()
        mine = {"k": int(res["k"]), "f_hist": [float(v) for v in res["f_hist"]],
                "fval": float(res["fval"]), "x_sha": hashlib.sha256(x.tobytes()).hexdigest(),
                "stats": [float(v) for v in res["stats"]], "syncs": int(res["syncs"])}
        got = [None] * world
        dist.all_gather_object(got, mine)
        runs[str(w)] = got
    if rank == 0:
        with open(a.out, "w") as fh:
            json.dump(runs, fh)
    comm.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
