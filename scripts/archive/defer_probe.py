"""Round 5 probe: ProxGD / FProxGD whole solves on a line-search-heavy instance (alpha0 x SCALE:
rejected first trials, so packets are published by k_publish(_pub) rather than carried by the
speculative kernel), iterations/s with the current GLX_DEFER_RED. Run under rocprofv3 to see the
publish kernels' durations."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "convex-optimization_amd"))
import torch  # noqa: E402
import glx  # noqa: E402
from oracle import numpy_ref  # noqa: E402

method = sys.argv[1] if len(sys.argv) > 1 else "gl_ProxGD_primal"
scale = float(sys.argv[2]) if len(sys.argv) > 2 else 2.5
m, n, l = 2048, 8192, 32
A, b, u, x0, mu = numpy_ref.gen_data(m, n, l, 3)
At, bt = torch.from_numpy(A).cuda(), torch.from_numpy(b).cuda()
opts = {"alpha0": scale * numpy_ref.step_size_for(m, n), "maxit": 300}
x, k, out = glx.solve(method, torch.from_numpy(x0).cuda(), At, bt, mu, dict(opts))   # warm
x, k, out = glx.solve(method, torch.from_numpy(x0).cuda(), At, bt, mu, dict(opts))
print(json.dumps({"method": method, "scale": scale, "defer": os.environ.get("GLX_DEFER_RED", "1"),
                  "k": int(k), "it_s": k / out["tt"], "syncs": out["glx"]["syncs"],
                  "fval": float(out["fval"])}), flush=True)
