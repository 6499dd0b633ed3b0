"""Per-piece timeline of the screened closure's refine pass (CDX_DIAG_WGTIME build): for each of the
256 pieces its duration, segment count and K-steps — whether pieces with more segments (more
prologue / epilogue / partial-tile stores) finish later.

  CDX_LIB=compliancedex_amd/lib/libcdx_wgtime.so python tools/refine_pieces.py     (GPU)
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    from compliancedex_amd import ProbabilisticGraspOptimizer
    from compliancedex_amd import _native as N
    from compliancedex_amd.urdf import load_robot
    from compliancedex_amd.workloads import prob_inputs, synthetic_banana_gpis
    cfg = load_robot("allegro")["config"]
    g = synthetic_banana_gpis(2000, device="cuda")
    E = 4096
    q, comp, target, palm = prob_inputs(cfg["ref_q"], E, seed=1000, spread=True)
    opt = ProbabilisticGraspOptimizer("allegro", cfg["ee_link_name"], cfg["ee_link_offset"], palm_offset=palm,
                                      ref_q=cfg["ref_q"], optimize_target=True, optimize_palm=True, device="cuda")
    t = [torch.from_numpy(np.ascontiguousarray(a)).cuda().requires_grad_(True)
         for a in (q, comp, target, palm[:, :3], palm[:, 3:])]
    for _ in range(5):
        opt.closure(*t, 1, g, E)
    torch.cuda.synchronize()
    lib = N.load()
    lib.cdx_diag_wgtime.argtypes = [ctypes.c_void_p, ctypes.c_int]
    buf = np.zeros((256, 4), dtype=np.uint64)
    assert lib.cdx_diag_wgtime(buf.ctypes.data, 256) == 0
    t0 = buf[:, 0].min()
    st, en = (buf[:, 0] - t0) / 100.0, (buf[:, 1] - t0) / 100.0  # 100 MHz ticks -> us
    seg = (buf[:, 3] >> 32).astype(int)
    ks = (buf[:, 3] & 0xffffffff).astype(int)
    dur = en - st
    out = {"pieces": 256, "start_us": [float(st.min()), float(st.max())], "end_us": [float(en.min()), float(en.max())],
           "dur_us_median": float(np.median(dur)), "ksteps": [int(ks.min()), int(ks.max())]}
    for n in sorted(set(seg)):
        m = seg == n
        out[f"segments_{n}"] = {"pieces": int(m.sum()), "dur_us_mean": float(dur[m].mean()), "end_us_mean": float(en[m].mean())}
    np.save(os.path.join(REPO, "gpurun_out", "refine_pieces.npy"), buf)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
