"""One call of glx_residual_gradient2 at a shape, with per-output error figures (debug aid)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "convex-optimization_amd"))
import torch  # noqa: E402
from glx import kernels  # noqa: E402

m, n = int(sys.argv[1]), int(sys.argv[2])
A = torch.randn(m, n, device="cuda", dtype=torch.float64)
X0 = torch.randn(n, 16, device="cuda", dtype=torch.float64)
X1 = torch.randn(n, 16, device="cuda", dtype=torch.float64)
B = torch.randn(m, 16, device="cuda", dtype=torch.float64)
for rep in range(2):
    R0, R1, G, ran = kernels.residual_gradient2(A, X0, X1, B, one_pass=True)
    torch.cuda.synchronize()
    e0 = float((R0 - (A @ X0 - B)).abs().max())
    e1 = float((R1 - (A @ X1 - B)).abs().max())
    Gr = A.T @ R1
    nan = int((~torch.isfinite(G)).sum())
    bad_rows = (~torch.isfinite(G)).any(1).nonzero().flatten()
    eg = float((torch.nan_to_num(G, nan=0.0) - Gr).abs().max())
    print(f"m={m} n={n} rep={rep} ran={ran} errR0={e0:.3e} errR1={e1:.3e} G_nonfinite={nan} "
          f"bad_rows={bad_rows[:8].tolist()} errG(finite)={eg:.3e} |G|max={float(Gr.abs().max()):.3e}",
          flush=True)
