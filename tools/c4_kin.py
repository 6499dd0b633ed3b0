"""Config 4's SDF / Kin leg on the GPU: the fused KinGraspOptimizer loop (workloads.config4_kin_inputs, E = 16 384
iiwa7_allegro candidates, 16 384-face banana) — ms per iteration (HIP events), the TorchSDF work counters, and
the same for round 4's timed workload ('far': arm base at the origin, q = 0.3·N(0, 1)).

  python tools/c4_kin.py [ITERS] [REPS] [around,far]
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(kind, iters, reps):
    import ctypes
    from compliancedex_amd import KinGraspOptimizer
    from compliancedex_amd import _native as N
    from compliancedex_amd.workloads import banana_mesh, config4_kin_inputs
    dev = "cuda"
    E = 16384
    links, offs, palm, q, target, comp = config4_kin_inputs(E, device=dev, q_scale=0.05 if kind == "around" else 0.3)
    if kind == "far":
        palm = palm * 0
    kin = KinGraspOptimizer("iiwa7_allegro", links, offs, palm_offset=palm.tolist(), num_iters=iters,
                            optimize_target=True, ref_q=[0.0] * 23)
    args = [torch.from_numpy(a).to(dev) for a in (q, target, comp)]
    mesh = banana_mesh()
    import copy
    kin.optimize(*args, 1, copy.deepcopy(mesh), verbose=False)  # warm-up (mesh prepare, allocator)
    torch.cuda.synchronize()
    ms, loop = [], []
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for _ in range(reps):
        m = copy.deepcopy(mesh)
        kin.loop_events = ev  # the iterations alone (HIP events on the loop's stream), as bench.py's config4_kin
        t0 = time.perf_counter()
        kin.optimize(*args, 1, m, verbose=False)
        torch.cuda.synchronize()
        ms.append((time.perf_counter() - t0) * 1e3 / iters)  # the whole call: mesh preparation (host k-d) included
        loop.append(ev[0].elapsed_time(ev[1]) / iters)
    kin.loop_events = None
    lib = N.load()
    st = (ctypes.c_uint64 * 3)()
    visits = ctypes.c_uint64(0)
    N.check(lib.cdx_sdf_stats(1, None, N.stream_ptr(dev)), "stats")
    kin.optimize(*args, 1, copy.deepcopy(mesh), verbose=False)
    N.check(lib.cdx_sdf_stats(0, st, N.stream_ptr(dev)), "stats")
    N.check(lib.cdx_sdf_chunk_visits(ctypes.byref(visits), N.stream_ptr(dev)), "visits")
    calls = max(1, int(st[2]) // (4 * E))
    print(json.dumps({"case": f"config4_kin_{kind}", "E": E, "iterations": iters, "ms_per_iteration_host": ms,
                      "ms_per_iteration_loop": loop, "min_ms": min(loop), "min_ms_host": min(ms),
                      "evals_per_s": E / (min(loop) * 1e-3), "sdf_calls": calls,
                      "pairs_per_call": int(st[0]) / calls, "pairs_exact_per_call": int(st[1]) / calls,
                      "pairs_per_point": int(st[0]) / max(1, int(st[2])),
                      "chunk_visits_per_wave": int(visits.value) / max(1, int(st[2]) // 64)}), flush=True)


if __name__ == "__main__":
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    kinds = sys.argv[3].split(",") if len(sys.argv) > 3 else ["around", "far"]
    for kind in kinds:
        run(kind, iters, reps)
