"""Margins of the HIP fp32 FProxGD whole solve at C3 against the reference's run
(tests/golden/c3_gl_FProxGD_primal.npz): k, fval and f_hist relative differences, for the
default (the dense batch) and the opt-in split-candidate batch (GLX_SPLIT_F32=1). One JSON line
per mode."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODE = r'''
import json, os, sys
import numpy as np
sys.path.insert(0, %(root)r); sys.path.insert(0, os.path.join(%(root)r, "convex-optimization_amd"))
import torch
from oracle import numpy_ref
G = os.path.join(%(root)r, "tests", "golden")
meta = json.load(open(os.path.join(G, "c3_gl_FProxGD_primal.json")))
A, _, u, x0, mu = numpy_ref.gen_data(meta["m"], meta["n"], meta["l"], meta["seed"])
b = np.load(os.path.join(G, "ns_instance_b.npz"))["b"]
A32, b32, x032 = (a.astype(np.float32) for a in (A, b, x0)); del A
gold = np.load(os.path.join(G, "c3_gl_FProxGD_primal.npz"))
from gl_FProxGD_primal import gl_FProxGD_primal
x, k, out = gl_FProxGD_primal(torch.from_numpy(x032).cuda(), torch.from_numpy(A32).cuda(),
                              torch.from_numpy(b32).cuda(), mu, dict(meta["opts"]))
fh = np.asarray([float(v) for v in out["f_hist"]]); fg = gold["f_hist"]; n = min(len(fh), len(fg))
rel = np.abs(fh[:n] - fg[:n]) / np.abs(fg[:n])
xr = gold["x"].astype(np.float64); xx = x.cpu().numpy().astype(np.float64)
print(json.dumps({"mode": os.environ.get("MODE"), "k": int(k), "k_ref": int(gold["k"]),
                  "fval_rel": abs(float(out["fval"]) - float(gold["fval"])) / abs(float(gold["fval"])),
                  "fhist_rel_max": float(rel.max()), "fhist_rel_last": float(rel[-1]),
                  "x_err_over_max": float(np.max(np.abs(xx - xr)) / np.max(np.abs(xr)))}), flush=True)
''' % {"root": ROOT}
MODES = [("split", {"GLX_SPLIT_F32": "1"}), ("dense", {})]
if "--variants" in sys.argv:   # other summation orders of the same two forms (noise draws)
    MODES = [("dense_S4", {"GLX_AXB_S": "4"}), ("dense_S16", {"GLX_AXB_S": "16"}),
             ("dense_52224", {"GLX_AXB_VARIANT": "52224"}),
             ("split_21410", {"GLX_SPLIT_F32": "1", "GLX_AX_DMA32": "0"}),
             ("split_S4", {"GLX_SPLIT_F32": "1", "GLX_AX_S": "4"})]
for mode, env in MODES:
    e = dict(os.environ, MODE=mode, **env)
    r = subprocess.run([sys.executable, "-c", CODE], env=e, capture_output=True, text=True, timeout=600)
    sys.stdout.write(r.stdout)
    if r.returncode != 0:
        sys.stderr.write(r.stderr[-3000:])
        sys.exit(r.returncode)
