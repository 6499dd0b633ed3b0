"""Where kin_cost4_kernel<16, true, true>'s time goes: per-wave shader-clock stamps at its phases (a timing-only
CDX_KIN_DIAG_PHASES build, lib/libcdx_kphase.so), last iteration of a config-4 fused Kin loop, median over waves.

  python tools/kin_phases.py build     # (CPU) the diagnostic library
  python tools/kin_phases.py run       # (GPU)
"""
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PHASES = ["gather + DMA issue", "reward forward (Kabsch SVD, equilibrium)", "cost forward", "cost + reward backward",
          "FK backward (+ sums)", "step (best iterate, Adam)", "next fingertips (FK walk)"]


def main():
    if sys.argv[1] == "build":
        from compliancedex_amd.build import DEFAULT_DEFINES, build_device
        build_device(force=True, defines=tuple(DEFAULT_DEFINES) + ("CDX_KIN_DIAG_PHASES",), out_name="libcdx_kphase.so")
        return
    os.environ["CDX_LIB"] = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "compliancedex_amd",
                                         "lib", "libcdx_kphase.so")
    import torch
    from compliancedex_amd import KinGraspOptimizer
    from compliancedex_amd import _native as N
    from compliancedex_amd.workloads import banana_mesh, config4_kin_inputs
    E = 16384
    links, offs, palm, q, target, comp = config4_kin_inputs(E, device="cuda", q_scale=0.05)
    out = {}
    for cache in ("1", "0"):
        os.environ["CDX_KIN_FK_CACHE"] = cache
        kin = KinGraspOptimizer("iiwa7_allegro", links, offs, palm_offset=palm.tolist(), num_iters=12,
                                optimize_target=True, ref_q=[0.0] * 23)
        args = [torch.from_numpy(a).to("cuda") for a in (q, target, comp)]
        kin.optimize(*args, 1, banana_mesh(), verbose=False)
        torch.cuda.synchronize()
        lib = N.load()
        buf = (ctypes.c_uint64 * (4096 * 16))()
        assert lib.cdx_kin_phase_read(buf) == 0
        t = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 16)[:4 * E // 64].astype(np.int64)
        d = np.diff(t[:, :8], axis=1)
        tot = t[:, 7] - t[:, 0]
        sub = {"bwd: prefetch issue": t[:, 12] - t[:, 4], "bwd: wait + check": t[:, 13] - t[:, 12],
               "bwd: grad": t[:, 14] - t[:, 13], "bwd: sums": t[:, 5] - t[:, 14], "syncthreads": t[:, 11] - t[:, 6], "to walk": t[:, 8] - t[:, 11], "walk3r": t[:, 9] - t[:, 8],
               "pose + stores": t[:, 10] - t[:, 9], "tips": t[:, 7] - t[:, 10]} if cache == "1" else {}
        out[f"cache{cache}"] = {"wave_cycles_median": float(np.median(tot)),
                                "phases_median_cycles": {PHASES[i]: float(np.median(d[:, i])) for i in range(7)},
                                "phases_share": {PHASES[i]: float(np.median(d[:, i]) / np.median(tot)) for i in range(7)},
                                "writer_median_cycles": {k: float(np.median(v)) for k, v in sub.items()}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
