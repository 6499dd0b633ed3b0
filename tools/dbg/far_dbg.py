import numpy as np, torch
from compliancedex_amd.workloads import synthetic_banana_gpis, prob_inputs
from compliancedex_amd.gpis import exact_var
from tests.test_screen import _all_tip_queries, _opt
g = synthetic_banana_gpis(2000, device="cuda")
st = g.native_state()
print("R", float(g.R), "delta/k0", st.desc.screen_delta / float(g.R) ** 3, "err/k0", st.screen_err / float(g.R) ** 3)
sc = st.screen.view(torch.float64)
cfg, opt = _opt()
q, comp, target, palm = prob_inputs(cfg["ref_q"], 2048, seed=99, spread=True)
palm = palm.copy(); palm[:128, 0] += 2.0
from oracle.cdx_oracle import OracleChain, OracleProblem
from compliancedex_amd.urdf import load_robot
prob = OracleProblem(OracleChain(load_robot("allegro")["bodies"]), cfg["ee_link_name"], cfg["ee_link_offset"], cfg["ref_q"], None)
with torch.no_grad():
    pre = prob.forward_kinematics(torch.from_numpy(q), torch.from_numpy(palm)).double()
tgt = torch.from_numpy(target)
X = (tgt + 0.8 * (pre - tgt)).reshape(-1, 3).cuda()
est = st.screen_var(X); ex = exact_var(st, X)
c = g.X1.double().mean(0)
dist = (X - c).norm(dim=1)
err = (est - ex).abs()
bad = torch.isfinite(est) & (err > st.desc.screen_delta)
k0 = float(g.R) ** 3
print("nan rows", int((~torch.isfinite(est)).sum()), "bad", int(bad.sum()))
idx = torch.nonzero(bad).flatten()[:20]
for i in idx.tolist():
    print(i, "dist", float(dist[i]), "est/k0", float(est[i]) / k0, "ex/k0", float(ex[i]) / k0)
fin = torch.isfinite(est)
print("max dist finite", float(dist[fin].max()), "min dist nan", float(dist[~fin].min()) if (~fin).any() else None)
