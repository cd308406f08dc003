"""Benchmark: proximal-gradient iterations/s on (m,n,l) = (8192,16384,32) fp64 (BASELINE.json).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--method gl_ProxGD_primal] [--dtype f64]
                    [--m 8192 --n 16384 --l 32] [--no-cpu-baseline] [--variant V]

One step = one recorded iteration of the solver (objective, stop rule, threshold, A^T(Ax-b),
line search, prox) on one synthetic instance whose A, b, x live in HBM before timing starts.
N > 1 (one process per GPU): A and b are row-sharded, the gradient is summed with RCCL, and
the same global problem is solved (strong scaling); the reported value is iterations/s of the
whole job (max of the per-rank times). Launched either by torch.distributed.run (RANK /
WORLD_SIZE set), or as plain `python bench.py --gpus N`: then this process touches no GPU, starts
`torch.distributed.run --nproc-per-node N` on itself as a child and exits with its code (rank 0
prints the JSON line). Fewer than N visible devices, or a launcher world size that differs
from --gpus, is an error (exit 2), never a silent one-rank measurement.

Pre-warm (outside the timed region, declared in the line as `prewarm`): before the W warmup
steps every rank runs a throwaway solver session on the same instance for --prewarm-s seconds
(default 0.5). After ~1 s idle the MI355X's power management lets the first ~2 ms of fp64 MFMA
load run fast, then throttles (A@X 290 -> 400+ us) and recovers over ~30 ms
(profiles/r2_power_probe.jsonl); a 20-step run would otherwise time that transient, not the
solver. The timed session restarts from x0, so the iterations timed are the same ones.

Also reported, for the dominant kernel (round 4: whichever of the two passes over A — the dense
A@X pass or the fused A^T r + trial — has the longer average launch; at NS that is A^T r, ~43 %
of the iteration, with A@X a few us behind):
  roofline — the kernel's bound is whichever of MFMA time (flops / dense MFMA peak) and HBM time
             (bytes / 8 TB/s) is larger for this (m, n, l, dtype) and right-hand-side count: HBM
             at NS (one right-hand side: l/4 flop/B in fp64, 109 us of MFMA against 135 us of HBM),
             at C2 and for C4 (l = 1); MFMA for the batched two-source passes (FProxGD's dense
             batches, C3 in fp32). achieved =
             algorithmic flops 2*m*n*l*rhs (or bytes s*(m n + (m+n) l rhs)) per launch / average
             launch time from HIP events on every k-th dense A@X / A^T r launch of the timed
             region (--profile k, default min(16, steps/4)), attached to the kernel itself
             (hipExtLaunchKernel: the pair is stamped with that kernel's start and end on the
             solver's stream); `roofline.kernels` holds the same object for both passes (`ax`,
             `atr`), `roofline.dominant` names the one the top-level fields describe; the
             split-candidate A e gather is timed by its own pair and reported apart.
             `pair_frac` / `pair4_frac` are the same fraction for
             the A@x + A^T r pair (the north-star target), `pair4_frac_incl_gather` adds the
             gather. `traffic` = HBM bytes per launch from rocprofv3 PMC (profiles/pmc_traffic.json,
             2*FETCH_SIZE + WRITE_SIZE per the gfx950 correction) when that file holds the same
             config and kernel, else null;
  cpu_baseline — the repo's NumPy oracle (oracle/numpy_ref.py) on the host cores, on a bounded
             sample of the same instance (rank 0, N = 1 only).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "convex-optimization_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "prox-grad iters/sec + MFMA-roofline %, (m,n,l)=(8192,16384,32) fp64"
HBM_PEAK_GBS = 8000.0
MFMA_PEAK_TFS = {"f64": 78.6, "f32": 157.3}
BLOCK_ROWS = 256


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def make_instance(m, n, l, r0, r1, dtype, device, seed=97006855):
    """Large shapes (A beyond HOST_GEN_BYTES, e.g. C5's 131072 rows): A ~ N(0,1), a 10 % row-sparse
    ground truth u, b = A u, x0 ~ N(0,1), drawn with torch's Philox generator on the device per
    256-row block with per-block seeds, so every rank builds exactly its rows of the same global
    A. NOT the main.py:37-51 stream (the `data` label says so); no reference run exists for it."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    k = round(0.1 * n)
    u = torch.zeros(n, l, dtype=torch.float64, device=device)
    support = torch.randperm(n, generator=g, device=device)[:k]
    u[support] = torch.randn(k, l, generator=g, device=device, dtype=torch.float64)
    x0 = torch.randn(n, l, generator=g, device=device, dtype=torch.float64)
    A = torch.empty(r1 - r0, n, dtype=dtype, device=device)
    for blk in range(r0 // BLOCK_ROWS, (r1 + BLOCK_ROWS - 1) // BLOCK_ROWS):
        b0, b1 = blk * BLOCK_ROWS, min((blk + 1) * BLOCK_ROWS, m)
        g.manual_seed(seed * 1000003 + blk)
        rows = torch.randn(b1 - b0, n, generator=g, device=device, dtype=torch.float64)
        lo, hi = max(b0, r0), min(b1, r1)
        A[lo - r0:hi - r0] = rows[lo - b0:hi - b0].to(dtype)
        del rows
    b = (A.to(torch.float64) @ u).to(dtype)
    return A.contiguous(), b.contiguous(), x0.to(dtype).contiguous()


# The reference's own whole solves of the BASELINE configs (tests/golden/make_golden_*.py ran
# /root/reference/code on gen_data's instance in the build container): (method, dtype, m, n, l) ->
# (fixture stem, where b comes from). b = A u is taken from the fixture, because the host BLAS's
# A @ u is not portable bit for bit; A and x0 are re-drawn and sha256-checked against the fixture.
GOLDEN = {
    ("gl_ProxGD_primal", "f64", 8192, 16384, 32): ("ns_gl_ProxGD_primal", "ns_instance_b"),
    ("gl_FProxGD_primal", "f64", 8192, 16384, 32): ("ns_gl_FProxGD_primal", "ns_instance_b"),
    ("gl_FProxGD_primal", "f32", 8192, 16384, 32): ("c3_gl_FProxGD_primal", "ns_instance_b"),
    ("gl_ProxGD_primal", "f64", 4096, 8192, 16): ("c2_gl_ProxGD_primal", "c2_gl_ProxGD_primal"),
    ("gl_SGD_primal", "f64", 65536, 8192, 1): ("c4_gl_SGD_primal", "c4_gl_SGD_primal"),
}
GOLDEN_DIR = os.path.join(ROOT, "tests", "golden")
HOST_GEN_BYTES = 4.5 * 2 ** 30   # gen_data on the host up to this much fp64 A (C4: 4 GiB)


def _sha(a):
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def reference_instance(method, dt, m, n, l, r0, r1, dtype, device, seed=97006855):
    """The instance main.py:37-51 draws (gen_data: one MT19937(seed) stream, A, permutation, rows of
    u, x0 in that order; glx.driver.gen_data), generalised to (m, n, l); every rank draws the whole
    A on the host and keeps its rows [r0, r1). Where a reference whole solve of this exact call is
    committed (GOLDEN), b is that run's own A u and the line's whole_solve is checked against it.
    Returns (A, b, x0, info)."""
    from glx.driver import gen_data
    if m * n * 8 > HOST_GEN_BYTES:
        A, b, x0 = make_instance(m, n, l, r0, r1, dtype, device, seed)
        return A, b, x0, {"data": "synthetic, torch Philox on the device per 256-row block (A beyond "
                                  "%.1f GiB: main.py's MT19937 stream not drawn on the host); no "
                                  "reference run of this instance" % (HOST_GEN_BYTES / 2 ** 30),
                          "golden": None}
    _, _, _, _, An, bn, _, xn, _, _, _ = gen_data(seed, m, n, l)
    info = {"data": "synthetic: main.py:37-51 gen_data (MT19937 seed %d: A, permutation, u rows, x0) "
                    "at (m,n,l)=(%d,%d,%d), drawn on the host%s" % (seed, m, n, l,
                                                                    "" if dt == "f64" else ", cast to fp32"),
            "golden": None}
    key = GOLDEN.get((method, dt, m, n, l))
    if key is not None:
        stem, bsrc = key
        meta_p = os.path.join(GOLDEN_DIR, stem + ".json")
        if os.path.exists(meta_p):
            meta = json.load(open(meta_p))
            bref = np.load(os.path.join(GOLDEN_DIR, bsrc + ".npz"))["b"]
            if dt == "f64":
                ok = _sha(An) == meta["sha256"]["A"] and _sha(xn) == meta["sha256"]["x0"] and \
                    _sha(bref) == meta["sha256"]["b"]
            else:
                ok = _sha(An.astype(np.float32)) == meta["sha256"]["A32"] and \
                    _sha(xn.astype(np.float32)) == meta["sha256"]["x032"] and \
                    _sha(bref.astype(np.float32)) == meta["sha256"]["b32"]
            if ok:
                bn = bref
                info["golden"] = {"stem": stem, "meta": meta}
                info["data"] += ("; b = the reference run's own A u (tests/golden/%s.npz), A / x0 / b "
                                 "sha256 = tests/golden/%s.json" % (bsrc, stem))
            else:
                info["data"] += "; instance sha256 differs from tests/golden/%s.json: no reference check" % stem
    npdt = np.float64 if dt == "f64" else np.float32
    A = torch.from_numpy(np.ascontiguousarray(An[r0:r1], dtype=npdt)).to(device)
    b = torch.from_numpy(np.ascontiguousarray(bn[r0:r1], dtype=npdt)).to(device)
    x0 = torch.from_numpy(np.ascontiguousarray(xn, dtype=npdt)).to(device)
    return A, b, x0, info


def vs_reference(info, k, fval, f_hist, dt):
    """The whole solve against the committed reference run of the same call (GOLDEN): the
    north-star bar in fp64 (k identical, fval and every f_hist entry within 1e-8 relative); in
    fp32 SURVEY §8d's bar, as the C3 test (fval within 1e-6, k within 0.5 %)."""
    g = info.get("golden")
    if g is None:
        return None
    gold = np.load(os.path.join(GOLDEN_DIR, g["stem"] + ".npz"))
    kg, fg = int(gold["k"]), float(gold["fval"])
    fh = np.asarray(f_hist, dtype=np.float64)
    fh_rel = (float(np.max(np.abs(fh - gold["f_hist"]) / np.abs(gold["f_hist"])))
              if fh.shape == gold["f_hist"].shape else None)
    frel = abs(fval - fg) / abs(fg)
    if dt == "f64":
        ok = k == kg and frel <= 1e-8 and fh_rel is not None and fh_rel <= 1e-8
        bar = "k identical, fval and every f_hist entry within 1e-8 relative (north star, fp64)"
    else:   # C3 stops at maxit unconverged: its fp32 objective scatters with the summation order
        ok = frel <= 1e-6 and abs(k - kg) <= max(1, int(0.005 * kg))
        bar = ("fval within 1e-6 relative, k within 0.5 % (fp32, SURVEY §8d; "
               "tests/test_gpu_ns_golden.py::test_whole_solve_c3_fp32)")
    return {"reference": "tests/golden/%s.npz (the reference's own run of this call)" % g["stem"],
            "k_ref": kg, "k": int(k), "fval_ref": fg, "fval_rel_diff": frel,
            "f_hist_max_rel_diff": fh_rel, "bar": bar, "within_bar": bool(ok)}


def cpu_baseline(method, A, b, x0, mu, opts, budget_s=15.0):
    """Time the NumPy oracle (test infrastructure) on the host on a bounded sample: the same
    instance, a fixed number of iterations per continuation phase. The GPU solver then runs the
    same sample (same opts and maxit) and its f_hist is compared with the oracle's entry by entry
    (`gpu_same_sample`): parity evidence of the measured path inside the bench run itself."""
    from oracle import numpy_ref
    try:
        from threadpoolctl import threadpool_info
        info = [d for d in threadpool_info() if d.get("user_api") == "blas"]
        threads = int(info[0]["num_threads"]) if info else os.cpu_count()
        blas = "%s %s" % (info[0].get("internal_api"), info[0].get("version")) if info else "?"
    except Exception:
        threads, blas = os.cpu_count(), "?"
    An, bn, xn = A.cpu().numpy(), b.cpu().numpy(), x0.cpu().numpy()
    fn = numpy_ref.SOLVERS[method]
    # calibrate: one iteration per phase
    o = dict(opts, maxit=1)
    t0 = time.perf_counter()
    _, k1, _ = fn(xn, An, bn, mu, o)
    t1 = time.perf_counter() - t0
    per_iter = t1 / max(1, k1)
    maxit = int(max(1, min(200, budget_s / (3 * per_iter))))
    o = dict(opts, maxit=maxit)
    t0 = time.perf_counter()
    _, k, outc = fn(xn, An, bn, mu, o)
    dt = time.perf_counter() - t0
    import glx
    _, kg, outg = glx.solve(method, x0.clone(), A, b, mu, dict(o))
    fc = np.asarray([float(v) for v in outc["f_hist"]])
    fg = np.asarray([float(v) for v in outg["f_hist"]])
    same = {"k_cpu": int(k), "k_gpu": int(kg),
            "f_hist_max_rel_diff": (float(np.max(np.abs(fg - fc) / np.abs(fc)))
                                    if fg.shape == fc.shape else None),
            "fval_rel_diff": abs(float(outg["fval"]) - float(outc["fval"])) / abs(float(outc["fval"])),
            "what": "glx.solve on the same sample (maxit=%d per phase) against the oracle's run" % maxit}
    return {"value": k / dt, "unit": "iters/s", "cores": threads, "kind": "port",
            "sample": "oracle/numpy_ref.%s on the same instance, %d iterations (maxit=%d per phase), "
                      "%.1f s; BLAS %s" % (method, k, maxit, dt, blas),
            "gpu_same_sample": same}


PMC_FILE = "profiles/pmc_traffic.json"


def pmc_traffic(cfg_key, which="ax"):
    """(bytes per launch of the A@X pass (which="ax") or of the A^T r pass ("atr"), source) from
    the committed rocprofv3 PMC summary of a separate run of this same configuration
    (FETCH_SIZE / WRITE_SIZE passes cannot share the timed run); (None, None) when that file
    holds no entry for this configuration."""
    try:
        with open(os.path.join(ROOT, PMC_FILE)) as fh:
            d = json.load(fh)
        e = d.get(cfg_key)
        if e is None:
            return None, None
        v = e["bytes_per_launch"] if which == "ax" else e.get("detail", {}).get("atr", {}).get("bytes_per_launch")
        if v is None:
            return None, None
        return float(v), "%s[%s].%s (%s)" % (PMC_FILE, cfg_key, "bytes_per_launch" if which == "ax" else "detail.atr",
                                              e.get("source", "committed PMC run"))
    except Exception:
        return None, None


def roof_of(flops, nbytes, avg_s, peak_tf):
    """bound / achieved / peak / frac of one kernel from its algorithmic flops and bytes per
    launch and its average launch time"""
    mfma_bound = flops / (peak_tf * 1e12) >= nbytes / (HBM_PEAK_GBS * 1e9)
    tf = flops / avg_s / 1e12 if avg_s else None
    gbs = nbytes / avg_s / 1e9 if avg_s else None
    ach, peak, unit = (tf, peak_tf, "TFLOP/s") if mfma_bound else (gbs, HBM_PEAK_GBS, "GB/s")
    return {"bound": "mfma" if mfma_bound else "hbm", "achieved": ach, "peak": peak, "unit": unit,
            "frac": (ach / peak) if ach else None, "avg_launch_us": avg_s * 1e6 if avg_s else None,
            "flops_per_launch": flops, "bytes_per_launch": nbytes,
            "hbm_GBs": gbs, "hbm_frac": gbs / HBM_PEAK_GBS if gbs else None,
            "mfma_tflops": tf, "mfma_frac": tf / peak_tf if tf else None}


def launch_ranks(args):
    """`bench.py --gpus N` without a launcher: run torch.distributed.run with N processes on this
    script (one rank per GPU) as a CHILD process and return its exit code. Called before any GPU
    call; torch.cuda.device_count() does not initialise the GPU."""
    import socket
    import subprocess
    visible = torch.cuda.device_count()
    with socket.socket() as sk:          # a free rendezvous port on the loopback interface
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    argv = [a for a in sys.argv[1:] if a != "--dry-run-launch"]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node", str(args.gpus), "--master-addr", "127.0.0.1",
           "--master-port", str(port), os.path.abspath(__file__)] + argv
    ok = visible >= args.gpus or args.comm == "host"
    if args.dry_run_launch:
        print(json.dumps({"launch": cmd, "nproc": args.gpus, "visible_devices": visible, "ok": ok}))
        return 0
    if not ok:
        log("error: --gpus %d but only %d GPU(s) visible; refusing to measure fewer ranks" %
            (args.gpus, visible))
        return 2
    log("launching %d ranks: %s" % (args.gpus, " ".join(cmd)))
    return subprocess.call(cmd)


def glx_env():
    """Every GLX_* knob set in the environment (empty at the measured defaults)."""
    return {k: v for k, v in sorted(os.environ.items()) if k.startswith("GLX_")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--method", default="gl_ProxGD_primal")
    ap.add_argument("--dtype", default="f64", choices=["f64", "f32"])
    ap.add_argument("--m", type=int, default=8192)
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--l", type=int, default=32)
    ap.add_argument("--variant", type=int, default=0)
    ap.add_argument("--exact", type=int, default=0)
    ap.add_argument("--profile", type=int, default=None,
                    help="HIP events on every k-th A@x / A^T r / gather launch (0 = off; default: "
                         "min(16, steps // 4), so at least 4 launches of each are timed)")
    ap.add_argument("--prewarm-s", type=float, default=0.5,
                    help="seconds of a throwaway solver session before the warmup (0 = off)")
    ap.add_argument("--dry-run-launch", action="store_true",
                    help="print the launcher decision (child command, visible devices) and exit")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-whole-solve", action="store_true",
                    help="skip the whole-solve figure reported beside the timed window")
    ap.add_argument("--force-comm", action="store_true",
                    help="create the communicator even at world size 1 (runs the N-GPU code path "
                         "with identity all-reduces: a one-GPU model of a rank's schedule)")
    ap.add_argument("--shard-model", type=int, default=int(os.environ.get("GLX_SHARD_MODEL", "0")),
                    help="with --force-comm at world size 1: the per-rank timing model of G ranks of "
                         "the row-sharded ProxGD schedule (opts shard_model; every line-search test "
                         "accepted, so NOT a solve: the whole solve beside it runs without it)")
    ap.add_argument("--watchdog-s", type=float, default=None,
                    help="N > 1: per-rank deadline in seconds from the communicator's creation to the "
                         "end of the run (glx.watchdog: the diagnostic and the thread stacks to "
                         "stderr, then exit 3); default 300 (rccl) / 1500 (host), 0 = off")
    ap.add_argument("--comm", default="rccl", choices=["rccl", "host"],
                    help="N > 1 transport: rccl (one GPU per rank) or host (all ranks share "
                         "cuda:0, all-reduces staged through gloo — a one-GPU rehearsal, not a "
                         "performance number)")
    args = ap.parse_args()
    if args.profile is None:
        # a timed launch still costs ~11 us of queue gaps around it (profiles/r3_evt/): the
        # driver's 20-step form times 4 launches of each kind, not 10
        args.profile = max(1, min(16, args.steps // 4))

    if "WORLD_SIZE" not in os.environ and (args.gpus > 1 or args.dry_run_launch):
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log("error: the launcher started WORLD_SIZE=%d ranks but --gpus=%d" % (world, args.gpus))
        sys.exit(2)
    if args.comm == "host":
        local = 0
    elif local >= torch.cuda.device_count():
        log("error: LOCAL_RANK %d but only %d GPU(s) visible" % (local, torch.cuda.device_count()))
        sys.exit(2)
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)

    import glx
    from glx.dist import Comm, shard_rows
    dist = None
    comm = None
    if world > 1 or args.force_comm:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29512")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    wd = None
    if world > 1:
        # armed before the communicator exists: RCCL's bootstrap is a collective too
        from glx.watchdog import Watchdog
        dl = args.watchdog_s if args.watchdog_s is not None else (300.0 if args.comm == "rccl" else 1500.0)
        wd = Watchdog(dl, "bench.py (%s, %d ranks)" % (args.comm, world), rank=rank, world=world).start()
        wd.phase = "communicator bootstrap"
    if world > 1 or args.force_comm:
        comm = Comm.host_staged() if args.comm == "host" else Comm.from_torch_distributed()
        if wd is not None:
            wd.probe("communicator", comm.progress)

    m, n, l = args.m, args.n, args.l
    dtype = torch.float64 if args.dtype == "f64" else torch.float32
    r0, r1 = shard_rows(m, world, rank)
    t_gen = time.perf_counter()
    if wd is not None:
        wd.phase = "instance generation"
    A, b, x0, inst = reference_instance(args.method, args.dtype, m, n, l, r0, r1, dtype, device)
    torch.cuda.synchronize()
    log("rank %d: instance rows [%d,%d) x %d x %d %s generated in %.1fs (%s)" %
        (rank, r0, r1, n, l, args.dtype, time.perf_counter() - t_gen,
         "reference run %s" % inst["golden"]["stem"] if inst["golden"] else "no reference run"))
    mu = 1e-2
    alpha0 = float(1.0 / (math.sqrt(m) + math.sqrt(n)) ** 2)
    if inst["golden"] is not None:   # the reference run's own alpha0 (the same expression)
        alpha0 = float(inst["golden"]["meta"]["opts"]["alpha0"])
    total = args.warmup + args.steps
    opts = {"alpha0": alpha0, "maxit": max(total + 1, 2500), "max_total_iters": total,
            "profile": args.profile, "ax_variant": args.variant, "exact_objective": args.exact,
            "shard_model": args.shard_model if world == 1 else 0}
    prewarm = None
    # the timed session is created first (its workspace, A's transposed copy), so that its warmup
    # follows the pre-warm session's last iteration without the GPU idling in between (round 4:
    # after an idle gap the power management throttles the next few ms of fp64 MFMA load, and
    # the 20-step window times exactly that, profiles/r4_evt/)
    x = x0.clone()
    s = glx.Session(args.method, x, A, b, mu, opts, comm=comm)
    if wd is not None:
        wd.probe("timed session", s.progress)
        wd.phase = "pre-warm"
    pw = None
    if args.prewarm_s > 0:
        prewarm = {"seconds": args.prewarm_s, "iters": 0,
                   "what": "throwaway session of the same solver on the same instance before the "
                           "warmup, run right before it; the timed session starts from x0"}
        xw = x0.clone()
        pw = glx.Session(args.method, xw, A, b, mu, dict(opts, profile=0, max_total_iters=0),
                         comm=comm)
        if wd is not None:
            wd.probe("pre-warm session", pw.progress)
        t_pw = time.perf_counter()
        while True:
            got = pw.run(16)
            prewarm["iters"] += got
            # every rank must run the same number of chunks (each issues collectives): continue
            # only while the clock has time left on EVERY rank (min over ranks)
            go = torch.tensor([0 if (pw.finished or got == 0 or time.perf_counter() - t_pw >= args.prewarm_s)
                               else 1], dtype=torch.int64)
            if dist is not None:
                dist.all_reduce(go, op=dist.ReduceOp.MIN)
            if int(go.item()) == 0:
                break
        prewarm["seconds"] = round(time.perf_counter() - t_pw, 3)
        # closed before the timed warmup: only one session's workspace (with
        # its transposed copy of A) is live while timing; closing costs host time only
        pw.close()
        pw = None
        if wd is not None:
            wd.probe("pre-warm session", None)
    plan = s.describe()
    if wd is not None:
        wd.phase = "warmup and timed window"
    s.run(args.warmup)
    for kind in (0, 1, 2):
        s.kernel_time(kind)
    c0 = s.counters()

    if dist is not None:
        dist.barrier()
    # marker kernels (torch's spin kernel) around the timed region, outside it: they delimit the
    # timed launches in a rocprofv3 kernel trace of this command (scripts/prof_agree.py)
    torch.cuda._sleep(1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    done = s.run(args.steps)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    torch.cuda._sleep(1)
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        dist.barrier()
    c1 = s.counters()
    work = {k: c1[k] - c0[k] for k in c1}   # executed work of the timed region
    ax_n, ax_ms = s.kernel_time(0)
    atr_n, atr_ms = s.kernel_time(1)
    ga_n, ga_ms = s.kernel_time(2)
    res = s.finish()
    if wd is not None:
        wd.probe("timed session", None)
        wd.phase = "whole solve"
    s.close()
    if done != args.steps:
        log("warning: solver finished after %d of %d timed steps" % (done, args.steps))
    # Beside the K-step window (iterations warmup+1 .. warmup+K of the first continuation phase),
    # the complete solve from x0 to the solver's own stop rule, every rank (the same collectives),
    # timed by the solver itself (tt, synchronized): the split-candidate trials get slower later
    # in a solve (more rows flagged), so the window alone favours the start.
    whole = None
    if not args.no_whole_solve:
        wopts = {"alpha0": alpha0, "ax_variant": args.variant, "exact_objective": args.exact}
        _, kw, outw = glx.solve(args.method, x0.clone(), A, b, mu, wopts, comm=comm)
        torch.cuda.synchronize()
        whole = {"k": int(kw), "tt_s": float(outw["tt"]), "iters_per_s": float(kw) / float(outw["tt"]),
                 "fval": float(outw["fval"]),
                 "vs_reference": vs_reference(inst, int(kw), float(outw["fval"]), outw["f_hist"],
                                              args.dtype),
                 "what": "the whole continuation solve from x0 to the solver's stop rule (default "
                         "maxit), same instance and opts, timed by the solver (tt); not `value`"}

    if rank == 0:
        es = 8 if args.dtype == "f64" else 4
        ml = r1 - r0
        ax_avg_s = (ax_ms / max(1, ax_n)) / 1e3
        atr_avg_s = (atr_ms / max(1, atr_n)) / 1e3
        # dense right-hand sides batched per A@x launch (e.g. A @ [z | p_thr | p] in exact mode).
        # ProxGD's split-candidate mode: one dense pass A p_thr, and A e (e = p - p_thr, nonzero
        # only in the rows the hard threshold touched) gathered from the flagged rows of a
        # transposed copy of A (m values each); its algorithmic work is 2 m l flops per such row.
        nsrc = work["ax_sources"] / max(1, work["ax_calls"])
        # the split-candidate form the session runs (glx_session_describe: dense / the row form
        # k_at_rows / the column-list gather)
        parts = plan.split("; ")
        split_desc = next((q[6:] for q in parts if q.startswith("split=")), "dense")
        split_cand = split_desc != "dense"
        st = res["stats"]
        if args.method == "gl_ProxGD_primal" and split_cand:
            sparse_rows = st[1] / max(1.0, st[2])   # rows of e flagged per trial
            gather_rows = sparse_rows
        elif args.method == "gl_FProxGD_primal" and split_cand:
            # flagged rows (row form; VALU gather: nonzeros) of e_c per gathered batch; bytes
            # averaged over all trial batches (some are dense)
            sparse_rows = st[5] / max(1.0, st[3])
            gather_rows = st[5] / max(1.0, st[3] + st[4])
        else:
            sparse_rows, gather_rows = 0.0, 0.0
        # the dense A@X pass and the split-candidate gather are separate kernels, timed apart
        ax_bytes = es * (ml * n + (ml + n) * l * nsrc)
        ga_bytes = es * (n * l + ml * gather_rows) if split_cand else 0.0
        atr_bytes = es * (ml * n + (ml + n) * l)
        ax_flops = 2.0 * ml * n * l * nsrc
        ga_flops = 2.0 * ml * l * sparse_rows
        atr_flops = 2.0 * ml * n * l
        ga_avg_s = (ga_ms / ga_n) / 1e3 if ga_n else 0.0
        key = "ax%d=" % max(1, min(3, int(round(nsrc))))
        ax_kname = "A@X: " + next((q[len(key):] for q in parts if q.startswith(key)), "?")
        # PMC entries are keyed by configuration AND the A@X tile the planner picks, so a
        # measurement of another kernel is never reported as this one's traffic
        cfg_key = "%s_%s_%dx%dx%d_g%d|%s" % (args.method, args.dtype, m, n, l, world, ax_kname)
        peak_tf = MFMA_PEAK_TFS[args.dtype]
        pair_tf = ((ax_flops + atr_flops) / (ax_avg_s + atr_avg_s) / 1e12) if (ax_n and atr_n) else None
        # SURVEY §8d's literal pair: one A@x (l right-hand sides) + one A^T r = 4 m n l flops over
        # the same two launches (the batched second right-hand side is not counted)
        pair4_tf = ((4.0 * ml * n * l) / (ax_avg_s + atr_avg_s) / 1e12) if (ax_n and atr_n) else None
        # the same with the split-candidate gather's time (and flops) added to the pair
        pair4g_tf = (((4.0 * ml * n * l) + ga_flops) / (ax_avg_s + atr_avg_s + ga_avg_s) / 1e12
                     if (ax_n and atr_n) else None)
        traffic, traffic_src = pmc_traffic(cfg_key)
        atr_traffic, atr_traffic_src = pmc_traffic(cfg_key, "atr")
        # the A^T r panel and trial the session itself launches (glx_session_describe)
        atr_kname = "A^T r: " + next((q[4:] for q in parts if q.startswith("atr=")), "?")
        kernels = {"ax": dict(roof_of(ax_flops, ax_bytes, ax_avg_s if ax_n else None, peak_tf),
                              kernel=("k_gemv_pair_fused: A@[x|thr(x)] and A^T r in ONE pass over A (l = 1)"
                                      if work["atr_calls"] == 0 else ax_kname),
                              launches_timed=ax_n, traffic=traffic, traffic_source=traffic_src)}
        if work["atr_calls"] > 0:
            kernels["atr"] = dict(roof_of(atr_flops, atr_bytes, atr_avg_s if atr_n else None, peak_tf),
                                  kernel=atr_kname, launches_timed=atr_n, traffic=atr_traffic,
                                  traffic_source=atr_traffic_src)
        # the dominant kernel: the longer of the two passes
        dominant = "ax"
        if "atr" in kernels and atr_n and ax_n and atr_avg_s > ax_avg_s:
            dominant = "atr"
        dk = kernels[dominant]
        # every top-level per-kernel field describes the dominant kernel;
        # the other pass's are under kernels
        roof = {"bound": dk["bound"], "achieved": dk["achieved"], "peak": dk["peak"],
                "unit": dk["unit"], "frac": dk["frac"], "dominant": dominant,
                "traffic": dk["traffic"], "traffic_source": dk["traffic_source"], "pmc_key": cfg_key,
                "kernel": dk["kernel"], "kernels": kernels,
                "flops_per_launch": dk["flops_per_launch"],
                "bytes_per_launch": dk["bytes_per_launch"], "avg_launch_us": dk["avg_launch_us"],
                "launches_timed": dk["launches_timed"],
                "hbm_GBs": dk["hbm_GBs"], "hbm_frac": dk["hbm_frac"],
                "mfma_tflops": dk["mfma_tflops"], "mfma_frac": dk["mfma_frac"],
                "session_plan": plan,
                "timed_every": args.profile,
                "rhs_per_launch": nsrc,
                "split_candidate": split_desc if split_cand else False,
                "sparse_rows_per_launch": sparse_rows,
                "pair_tflops": pair_tf, "pair_frac": pair_tf / peak_tf if pair_tf else None,
                "pair_definition": "pair_frac: algorithmic MFMA flops of the dense A@X launch "
                                   "(2 m n l per dense right-hand side) + A^T r (2 m n l), over "
                                   "the two launches' time (HIP events around each kernel); the "
                                   "north-star 60 % target is read on this one. pair4_frac: "
                                   "SURVEY §8d's literal 4 m n l over the same time. "
                                   "pair4_frac_incl_gather: also counting the split-candidate A e "
                                   "gather kernel's time (and its 2 m l flops per flagged row)",
                "pair4_tflops": pair4_tf, "pair4_frac": pair4_tf / peak_tf if pair4_tf else None,
                "gather_avg_launch_us": ga_avg_s * 1e6 if ga_n else None, "gather_launches_timed": ga_n,
                "gather_bytes_per_launch": ga_bytes,
                "pair4_frac_incl_gather": pair4g_tf / peak_tf if pair4g_tf else None,
                # all MFMA flops issued in the timed region / its wall time (gaps, prox included)
                "iter_frac": (2.0 * ml * n * l * work["ax_sources"] + work["atr_calls"] * atr_flops
                              + ga_flops * work["ax_calls"])
                             / elapsed / 1e12 / peak_tf}
        steps = max(1, done)
        line = {
            "metric": METRIC, "value": steps / elapsed, "unit": "iters/s", "n_gpus": world,
            "steps": steps, "warmup": args.warmup, "ms_per_step": 1e3 * elapsed / steps,
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": args.dtype,
            "data": inst["data"],
            "config": {"workload": "%s %s (m,n,l)=(%d,%d,%d), mu0=1e-2, alpha0=1/(sqrt(m)+sqrt(n))^2"
                                   % (args.method, args.dtype, m, n, l, ),
                       "method": args.method, "m": m, "n": n, "l": l,
                       "parallelism": ("row-shard x%d (%s; %s)" % (
                                           world, "RCCL" if args.comm == "rccl" else "host-staged gloo, ranks sharing one GPU",
                                           "reduce-scatter of A^T r, trial on n/%d rows, all-gather of p" % world
                                           if "rows=sharded" in plan else "all-reduce of A^T r"))
                                       if world > 1 else "single GPU",
                       "exact_objective": args.exact, "ax_variant": args.variant,
                       "timing_model": ("per-rank timing model of %d ranks (opts shard_model): "
                                        "every line-search test accepted, value is NOT a solve's rate"
                                        % args.shard_model) if (world == 1 and args.shard_model > 1
                                                                 and "timing model" in plan) else None},
            "roofline": roof,
            "prewarm": prewarm,
            "whole_solve": whole,
            "env": glx_env(),
            "work": {"ax_per_iter": work["ax_calls"] / steps, "atr_per_iter": work["atr_calls"] / steps,
                     "passes_over_A_per_iter": (work["ax_calls"] + work["atr_calls"]) / steps,
                     "syncs_per_iter": work["syncs"] / steps,
                     "thr_changed_entries_per_step": res["stats"][0] / max(1.0, res["stats"][2]),
                     "thr_changed_rows_per_step": res["stats"][1] / max(1.0, res["stats"][2]),
                     "syncs_total": res["syncs"], "iters_total": res["k"],
                     # ProxGD line-search decisions taken on the device (solver.cpp dc_run)
                     "device_decided_frac": (res["stats"][7] / max(1, res["k"])
                                             if args.method == "gl_ProxGD_primal" else 0.0)},
        }
        if world == 1 and not args.no_cpu_baseline:
            try:
                line["cpu_baseline"] = cpu_baseline(args.method, A, b, x0, mu,
                                                    {"alpha0": alpha0})
            except Exception as e:  # report, never fake
                line["cpu_baseline"] = {"value": None, "error": repr(e)}
        print(json.dumps(line), flush=True)
    if wd is not None:
        wd.stop()
    if comm is not None:
        comm.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
