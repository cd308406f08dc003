"""Sample board power and clocks with amd-smi while NS ProxGD solves run back to back.

    python scripts/power_sample.py --seconds 10 --out gpurun_out/x/power.jsonl [GLX_* env as usual]

Diagnostic for VERDICT round 3 weak item 2 (is the steady-state NS iteration power-limited?).
One JSON line per amd-smi sample; the solver loop's it/s goes on the last line.
"""
import argparse
import json
import os
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "convex-optimization_amd"))
sys.path.insert(0, ROOT)


def sampler(stop, out, period):
    while not stop.is_set():
        t = time.time()
        try:
            r = subprocess.run(["amd-smi", "metric", "-g", "0", "--power", "--clock", "--json"],
                               capture_output=True, text=True, timeout=5)
            rec = {"t": t, "rc": r.returncode, "out": r.stdout[:200000], "err": r.stderr[-300:]}
        except Exception as e:  # report, never fake
            rec = {"t": t, "error": repr(e)}
        out.write(json.dumps(rec) + "\n")
        out.flush()
        stop.wait(period)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--period", type=float, default=0.5)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    import math
    import torch
    import bench
    import glx
    torch.cuda.set_device(0)
    m, n, l = 8192, 16384, 32
    A, b, x0 = bench.make_instance(m, n, l, 0, m, torch.float64, torch.device("cuda", 0))
    alpha0 = 1.0 / (math.sqrt(m) + math.sqrt(n)) ** 2
    out = open(a.out, "w")
    stop = threading.Event()
    th = threading.Thread(target=sampler, args=(stop, out, a.period), daemon=True)
    th.start()
    t0 = time.perf_counter()
    iters = 0
    while time.perf_counter() - t0 < a.seconds:
        _, k, o = glx.solve("gl_ProxGD_primal", x0.clone(), A, b, 1e-2, {"alpha0": alpha0})
        iters += int(k)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    stop.set()
    th.join(timeout=10)
    out.write(json.dumps({"iters": iters, "seconds": dt, "iters_per_s": iters / dt}) + "\n")
    out.close()
    print("power sampling done: %.1f it/s" % (iters / dt))


if __name__ == "__main__":
    main()
