"""C3 (gl_FProxGD_primal fp32, (8192, 16384, 32), the reference's gen_data instance cast to fp32)
whole solves under several summation orders of each batch form: the
dense [xc | y_next] batch and the split-candidate batch (GLX_SPLIT_F32=1), each with its planner
default and other K splits / tiles / A e forms. Per variant: k, the final objective's relative
distance to the reference's own fp32 run (tests/golden/c3_gl_FProxGD_primal.npz) and to its fp64
run of the same instance (ns_gl_FProxGD_primal.npz: the exact-arithmetic target the fp32 runs
approximate), the last f_hist entry's distance, and the whole solve's iterations/s. One process
per variant (the GLX_* knobs some launchers read once per process). One JSON line each."""
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
import bench
G = os.path.join(%(root)r, "tests", "golden")
A, b, x0, info = bench.reference_instance("gl_FProxGD_primal", "f32", 8192, 16384, 32, 0, 8192,
                                          torch.float32, torch.device("cuda", 0))
assert info["golden"] is not None, info["data"]
g32 = np.load(os.path.join(G, "c3_gl_FProxGD_primal.npz"))
g64 = np.load(os.path.join(G, "ns_gl_FProxGD_primal.npz"))
import glx
x, k, out = glx.solve("gl_FProxGD_primal", x0.clone(), A, b, 1e-2, dict(info["golden"]["meta"]["opts"]))
fv = float(out["fval"]); fh = np.asarray([float(v) for v in out["f_hist"]])
r = lambda a, ref: abs(a - ref) / abs(ref)
print(json.dumps({"variant": os.environ.get("VARIANT"), "k": int(k), "it_s": k / out["tt"],
                  "fval": fv, "fval_rel_ref32": r(fv, float(g32["fval"])),
                  "fval_rel_ref64": r(fv, float(g64["fval"])),
                  "fhist_last_rel_ref32": r(fh[-1], float(g32["f_hist"][-1])),
                  "ref32_vs_ref64": r(float(g32["fval"]), float(g64["fval"]))}), flush=True)
''' % {"root": ROOT}
VARIANTS = [
    ("dense", {}), ("dense_axbS4", {"GLX_AXB_S": "4"}), ("dense_axbS16", {"GLX_AXB_S": "16"}),
    ("dense_52224", {"GLX_AXB_VARIANT": "52224"}), ("dense_atrS2", {"GLX_ATR_S": "2"}),
    ("split", {"GLX_SPLIT_F32": "1"}), ("split_axS4", {"GLX_SPLIT_F32": "1", "GLX_AX_S": "4"}),
    ("split_axS16", {"GLX_SPLIT_F32": "1", "GLX_AX_S": "16"}),
    ("split_21410", {"GLX_SPLIT_F32": "1", "GLX_AX_DMA32": "0"}),
    ("split_rows", {"GLX_SPLIT_F32": "1", "GLX_GATHER": "rows"}),
    ("split_atrS2", {"GLX_SPLIT_F32": "1", "GLX_ATR_S": "2"}),
]
only = sys.argv[1:]
for name, env in VARIANTS:
    if only and name not in only:
        continue
    e = dict(os.environ, VARIANT=name, **env)
    p = subprocess.run([sys.executable, "-c", CODE], env=e, capture_output=True, text=True, timeout=300)
    sys.stdout.write(p.stdout)
    sys.stdout.flush()
    if p.returncode != 0:
        sys.stderr.write(p.stderr[-3000:])
        sys.exit(p.returncode)
