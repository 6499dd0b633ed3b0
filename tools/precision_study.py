"""Why the GPIS std GEMM stays in f64 (configs 4/5 name a bf16 / fp32 GPIS GEMM): std = sqrt|k0 − ‖L⁻¹k‖²|
with L⁻¹ and K* rounded to fp32 / bf16 (fp32 accumulate) vs f64, at near-surface and box queries of
the N = 2000 banana GPIS.  CPU only:  PYTHONPATH=. python tools/precision_study.py
"""
import numpy as np, torch, scipy.linalg as sl
from tests._helpers import oracle_gpis, rel_err
g = oracle_gpis("synthetic2000")
E = g.E11.numpy(); X1 = g.X1.numpy()
L = np.linalg.cholesky(E); Li = sl.solve_triangular(L, np.eye(len(E)), lower=True)
rng = np.random.default_rng(0)
# queries: near-surface points (surface samples + 5 mm noise) and random box points
surf = X1[14:14+1936]
Xs = surf[rng.choice(len(surf), 500)] + 0.005*rng.standard_normal((500,3))
lo, hi = X1.min(0)-0.02, X1.max(0)+0.02
Xb = lo + (hi-lo)*rng.random((500,3))
for name, Xq in (("near-surface", Xs), ("box", Xb)):
    k = g.k(g.X1, torch.from_numpy(Xq)).numpy()
    k0 = float(g.R)**3
    v = Li @ k; s64 = np.sqrt(np.abs(k0 - (v*v).sum(0)))
    for dt in (torch.float32, torch.bfloat16):
        Lt = torch.from_numpy(Li).to(dt); kt = torch.from_numpy(k).to(dt)
        vv = (Lt.float() @ kt.float()).double().numpy()
        s = np.sqrt(np.abs(k0 - (vv*vv).sum(0)))
        r = np.abs(s - s64)/s64
        print(name, dt, "std rel err median %.2e max %.2e" % (np.median(r), r.max()), "std range", s64.min(), s64.max())
