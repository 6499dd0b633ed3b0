"""Per-closure stream times of config 2 (bench.py's workload) over 40 closures, an idle pause, and 40 more — whether
the slower first closures of a process come back after the GPU idles (clock / power state) or not (one-time state).

  python tools/ramp_probe.py [PAUSE_S]
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(pause):
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

    host = []

    def run(n):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
        ev[0].record()
        for i in range(n):
            th = time.perf_counter()
            for t in ts:
                t.grad = None
            opt.closure(*ts, 1, gpis, E)
            ev[i + 1].record()
            host.append(round((time.perf_counter() - th) * 1e3, 3))
        torch.cuda.synchronize()
        return [round(ev[i].elapsed_time(ev[i + 1]), 3) for i in range(n)]

    a = run(40)
    time.sleep(pause)
    b = run(40)
    time.sleep(0.01)
    c = run(20)
    print(json.dumps({"pause_s": pause, "first": a, "after_pause": b, "after_10ms": c, "host_ms": host}), flush=True)


if __name__ == "__main__":
    main(float(sys.argv[1]) if len(sys.argv) > 1 else 2.0)
