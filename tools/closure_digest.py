"""Digest of the config-2 closure's outputs (bench.py's workload: E = 4096, the synthetic banana GPIS N = 2000,
Allegro) after a few closures, for bit-identity checks between library builds (CDX_LIB):

  CDX_LIB=.../libcdx_X.so python tools/closure_digest.py [CLOSURES]

prints one JSON line: sha256 of loss, margins and the five gradients (bytes), and the screen report's counts.
"""
import hashlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(n):
    from compliancedex_amd import ProbabilisticGraspOptimizer
    from compliancedex_amd.urdf import load_robot
    from compliancedex_amd.workloads import config3_gpis, prob_inputs
    dev = torch.device("cuda", 0)
    cfg = load_robot("allegro")["config"]
    E = 4096
    _, gpis = config3_gpis(0, dev, n_total=2000)
    q, comp, target, palm = prob_inputs(cfg["ref_q"], E, seed=1000, spread=True, center=None)
    opt = ProbabilisticGraspOptimizer("allegro", cfg["ee_link_name"], cfg["ee_link_offset"], palm_offset=palm,
                                      ref_q=cfg["ref_q"], optimize_target=True, optimize_palm=True, device=dev, seed=0)
    ts = [torch.from_numpy(a).to(dev).requires_grad_(True) for a in (q, comp, target, palm[:, :3], palm[:, 3:])]
    h = hashlib.sha256()
    for _ in range(n):
        for t in ts:
            t.grad = None
        opt.closure(*ts, 1, gpis, E)
        torch.cuda.synchronize()
        for t in [opt.total_loss, opt.total_margin] + [t.grad for t in ts]:
            h.update(t.detach().double().contiguous().cpu().numpy().tobytes())
    rep = opt.screen_stats(gpis, E) or {}
    print(json.dumps({"lib": os.environ.get("CDX_LIB", "default"), "closures": n, "sha256": h.hexdigest()[:32],
                      "screen": {k: (v if isinstance(v, (int, float)) else str(v)) for k, v in rep.items()}}), flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 3)
