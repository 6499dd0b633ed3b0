"""Per-closure GPU time over 300 back-to-back closures (config 2): shows the clock ramp a short
warm-up leaves in the timed region."""
import sys, json, time
sys.path.insert(0, "/root/repo")
import torch
from compliancedex_amd import ProbabilisticGraspOptimizer
from compliancedex_amd.urdf import load_robot
from compliancedex_amd.workloads import prob_inputs, synthetic_banana_gpis
dev = torch.device("cuda", 0)
cfg = load_robot("allegro")["config"]
E = 4096
gpis = synthetic_banana_gpis(2000, dev)
q, comp, target, palm = prob_inputs(cfg["ref_q"], E, seed=1000, spread=True)
opt = ProbabilisticGraspOptimizer("allegro", cfg["ee_link_name"], cfg["ee_link_offset"], palm_offset=palm,
                                  ref_q=cfg["ref_q"], optimize_target=True, optimize_palm=True, device=dev)
t = [torch.from_numpy(a).to(dev).requires_grad_(True) for a in (q, comp, target, palm[:, :3], palm[:, 3:])]
evs = []
for i in range(300):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for x in t: x.grad = None
    opt.closure(*t, 1, gpis, E)
    e1.record()
    evs.append((e0, e1))
torch.cuda.synchronize()
ms = [a.elapsed_time(b) for a, b in evs]
print(json.dumps({"per_closure_ms_first20": [round(x, 3) for x in ms[:20]],
                  "mean_by_50": [round(sum(ms[i:i+50]) / 50, 4) for i in range(0, 300, 50)]}))
