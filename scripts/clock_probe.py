"""Steady-state shader clock inside the two passes over A (diagnostic; needs the probe build).

    bash scripts/build_probe.sh          # builds abtree/probe with -DGLX_CLOCK_PROBE (CPU side)
    cd abtree/probe && python3 ../../scripts/clock_probe.py --steps 200 [--m .. --n .. --l ..]

Runs the NS ProxGD session (bench.py's instance, pre-warm, warmup) for --steps iterations back
to back, then reads the stamps the last A@X (k_ax_dma) and A^T R (k_atr_prox) launches left:
per workgroup Δs_memtime / Δs_memrealtime x 100 MHz = the clock its main loop ran at, and the
loop's wall time. MI355X_MICROARCH.md "DVFS give-back" (6).
"""
import argparse
import ctypes
import json
import math
import os
import sys
import time

sys.path.insert(0, os.path.join(os.getcwd(), "convex-optimization_amd"))
sys.path.insert(0, os.getcwd())

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--m", type=int, default=8192)
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--l", type=int, default=32)
    ap.add_argument("--method", default="gl_ProxGD_primal")
    ap.add_argument("--raw", default=None, help="also save the per-workgroup stamps (.npz)")
    ap.add_argument("--idle-ms", type=float, default=0.0,
                    help="sleep this long, then run one more iteration (a launch after idle)")
    a = ap.parse_args()
    import bench
    import glx
    from glx import _lib
    torch.cuda.set_device(0)
    m, n, l = a.m, a.n, a.l
    A, b, x0 = bench.make_instance(m, n, l, 0, m, torch.float64, torch.device("cuda", 0))
    alpha0 = 1.0 / (math.sqrt(m) + math.sqrt(n)) ** 2
    opts = {"alpha0": alpha0, "maxit": 100000, "max_total_iters": 0}
    pw = glx.Session(a.method, x0.clone(), A, b, 1e-2, dict(opts))
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.5:
        pw.run(16)
    pw.close()
    s = glx.Session(a.method, x0.clone(), A, b, 1e-2, dict(opts))
    s.run(a.warmup)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    s.run(a.steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if a.idle_ms > 0:
        time.sleep(a.idle_ms / 1e3)
        s.run(1)
        torch.cuda.synchronize()
    v = np.zeros((2, 2048, 12))
    for p, fn in ((0, "glx_probe_clock_ax"), (1, "glx_probe_clock_atr")):
        buf = (ctypes.c_ulonglong * (2048 * 12))()
        assert getattr(_lib.lib(), fn)(buf) == 0
        v[p] = np.frombuffer(buf, dtype=np.uint64).reshape(2048, 12).astype(np.float64)
    out = {"steps": a.steps, "iters_per_s": a.steps / dt, "idle_ms": a.idle_ms}
    if a.raw:
        np.savez_compressed(a.raw, stamps=v)
    for p, name in ((0, "ax_dma"), (1, "atr")):
        mt = v[p, :, 0::2]   # shader clock at stamps 0..3
        rt = v[p, :, 1::2]   # 100 MHz clock at stamps 0..3
        ok = (rt[:, 2] > rt[:, 1]) & (mt[:, 2] > mt[:, 1]) & (rt[:, 3] >= rt[:, 2]) & (rt[:, 0] > 0)
        if ok.sum() == 0:
            out[name] = None
            continue
        mt, rt = mt[ok], rt[ok]
        ghz = (mt[:, 2] - mt[:, 1]) / (rt[:, 2] - rt[:, 1]) * 0.1
        t0 = rt[:, 0].min()
        us = lambda a: a / 100.0
        q = lambda a: {"median": float(np.median(a)), "p10": float(np.percentile(a, 10)),
                       "p90": float(np.percentile(a, 90)), "max": float(a.max())}
        out[name] = {"blocks": int(ok.sum()), "clock_GHz": q(ghz),
                     "entry_offset_us": q(us(rt[:, 0] - t0)),
                     "prologue_us": q(us(rt[:, 1] - rt[:, 0])),
                     "loop_us": q(us(rt[:, 2] - rt[:, 1])),
                     "epilogue_us": q(us(rt[:, 3] - rt[:, 2])),
                     "end_offset_us": q(us(rt[:, 3] - t0)),
                     "span_us": float(us(rt[:, 3].max() - t0))}
        if p == 1 and (rt[:, 4] > 0).all():
            out[name]["lds_reduce_us"] = q(us(rt[:, 4] - rt[:, 2]))
            out[name]["rows_us"] = q(us(rt[:, 5] - rt[:, 4]))
            out[name]["grid_reduce_us"] = q(us(rt[:, 3] - rt[:, 5]))
    s.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
