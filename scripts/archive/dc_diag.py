"""Diagnostic: host vs device-controlled ProxGD on one case; first differing record."""
import os, sys
sys.path[:0] = [".", "convex-optimization_amd"]
import numpy as np
import torch
import glx
from oracle import numpy_ref

def run(win, shape, scale, opts):
    os.environ["GLX_DC_BATCH"] = str(win)
    A, b, u, x0, mu = numpy_ref.gen_data(*shape, 2024)
    o = {"alpha0": numpy_ref.step_size_for(shape[0], shape[1]) * scale}
    o.update(opts)
    At, bt, xt = (torch.from_numpy(a).cuda() for a in (A, b, x0))
    s = glx.Session("gl_ProxGD_primal", xt, At, bt, mu, o)
    s.run(0)
    r = s.finish()
    sp, ps, pb = s.trace()
    s.close()
    return xt.cpu().numpy(), r, ps, pb

for shape, scale, opts in [((256, 16384, 32), 1.0, {"maxit": 300}), ((512, 1024, 16), 1.0, {}),
                           ((512, 1024, 16), 2.5, {})]:
    xh, rh, psh, pbh = run(0, shape, scale, opts)
    xd, rd, psd, pbd = run(8, shape, scale, opts)
    fh, fd = np.array(rh["f_hist"]), np.array(rd["f_hist"])
    diff = np.nonzero(fh != fd)[0] if len(fh) == len(fd) else [-1]
    print(shape, scale, "k", rh["k"], rd["k"], "phases", psh, pbh, psd, pbd, "stats", rh["stats"], rd["stats"],
          "syncs", rh["syncs"], rd["syncs"], "ndiff", len(diff), "first", list(diff[:8]),
          "x equal", np.array_equal(xh, xd), flush=True)
    for i in list(diff[:4]):
        print("   i", i, repr(fh[i]), repr(fd[i]), flush=True)
