"""Config-4 TorchSDF forward as a profiling child: the three queries of one SDF/Kin iteration (4E fingertips vs
the deflated and the true 16 384-face banana — one point order for both — and 4E targets vs the true mesh;
E = 16 384, workloads.config4_kin_inputs) on prepared meshes, repeated REPS times; prints each query's mean time
(HIP events) and, with a CDX_SDF_DIAG library (CDX_LIB), the per-workgroup durations of the last launch.

  python tools/sdf_child.py [REPS] [around|far] [batch]   (under rocprofv3 --pmc / --kernel-trace; tools/pmc_sdf.sh)
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(reps, kind, batch=False):
    from compliancedex_amd import DifferentiableRobotModel, PreparedMesh
    from compliancedex_amd import _native as N
    from compliancedex_amd.optimizers import _face_vertices
    from compliancedex_amd.torchsdf import QueryWorkspace
    from compliancedex_amd.workloads import banana_mesh, config4_kin_inputs
    dev = "cuda"
    links, offs, palm, q, target, comp = config4_kin_inputs(16384, device=dev, q_scale=0.05 if kind == "around" else 0.3)
    if kind == "far":
        palm = palm * 0
    tips = (DifferentiableRobotModel("iiwa7_allegro", device=dev).compute_forward_kinematics(
        torch.from_numpy(q).to(dev), links, offsets=offs)[0].view(-1, 3) + torch.from_numpy(palm).to(dev)).contiguous()
    tg = torch.from_numpy(target).to(dev).view(-1, 3).contiguous()
    m = banana_mesh()
    faces = _face_vertices(m, dev)
    m.scale(0.9, center=[0, 0, 0])
    full, deflated = PreparedMesh(faces), PreparedMesh(_face_vertices(m, dev))
    ws_t, ws_g = QueryWorkspace(), QueryWorkspace()
    calls = [(deflated, tips, ws_t, False), (full, tips, ws_t, True), (full, tg, ws_g, False)]
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in calls]
    ms = [0.0] * len(calls)
    with torch.no_grad():
        for r in range(reps):
            for i, (mh, pt, w, ro) in enumerate(calls):
                ev[i][0].record()
                mh.query(pt, workspace=w, reuse_order=ro)
                ev[i][1].record()
            torch.cuda.synchronize()
            if r > 0:
                for i in range(len(calls)):
                    ms[i] += ev[i][0].elapsed_time(ev[i][1]) / (reps - 1)
    out = {"workload": kind, "query_ms": ms, "sum_ms": sum(ms)}
    nwg = (tg.shape[0] + 63) // 64
    if batch:  # the loop's batched launch (cdx_sdf_query_batch): its span, and the groups' timeline below
        from compliancedex_amd.torchsdf import BatchSchedule, query_batch
        sched = BatchSchedule() if os.environ.get("CDX_SDF_SCHED", "1") != "0" else None
        outs = [(torch.empty(p.shape[0], device=dev), torch.empty(p.shape[0], dtype=torch.int32, device=dev),
                 torch.empty(p.shape[0], 3, device=dev), torch.empty(p.shape[0], 3, device=dev))
                for p in (tips, tips, tg)]
        items = [(deflated, tips, ws_t, outs[0]), (full, tips, ws_t, outs[1]), (full, tg, ws_g, outs[2])]
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        bms = []
        for r in range(reps):
            e0.record()
            query_batch(items, schedule=sched)
            e1.record()
            torch.cuda.synchronize()
            bms.append(e0.elapsed_time(e1))
        out["batch_ms_min"], out["batch_ms_median"] = min(bms[1:] or bms), float(np.median(bms[1:] or bms))
        nwg = sum((p.shape[0] + 63) // 64 for p in (tips, tips, tg))
    lib = N.load()
    if hasattr(lib, "cdx_sdf_diag_wgtime"):
        import ctypes as C
        buf = np.zeros((nwg, 4), np.uint64)
        lib.cdx_sdf_diag_wgtime(buf.ctypes.data_as(C.c_void_p), C.c_int64(nwg), C.c_void_p(N.stream_ptr(dev)))
        t0 = buf[:, 0].min()
        start, end = (buf[:, 0] - t0) / 100.0, (buf[:, 1] - t0) / 100.0  # µs (100 MHz)
        dur = end - start
        vis, prs = buf[:, 2].astype(np.float64), buf[:, 3].astype(np.float64)
        slow = np.argsort(dur)[-8:]
        # the slow workgroups' points: spread (bbox diagonal) of their 64 sorted points
        order = ws_g.buf[:0]  # (placeholder: the order lives in the workspace; spread from the sorted targets)
        pts = tg.cpu().numpy()
        from compliancedex_amd import _native as _N  # noqa: F401
        if batch:  # per query of the batch: its groups' end times (where the launch's tail comes from)
            q_first = np.cumsum([0] + [(p.shape[0] + 63) // 64 for p in (tips, tips, tg)])
            out["batch_query_end_us"] = [[float(np.quantile(end[a:b], x)) for x in (0.5, 0.9, 0.99, 1.0)]
                                         for a, b in zip(q_first[:-1], q_first[1:])]
            out["batch_query_dur_us"] = [[float(np.quantile(dur[a:b], x)) for x in (0.5, 0.9, 0.99, 1.0)]
                                         for a, b in zip(q_first[:-1], q_first[1:])]
            np.save(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out",
                                 f"sdf_batch_wgtime_{kind}.npy"), buf)
        out["last_launch_wg_us"] = {"span": float(end.max()), "dur_p50": float(np.median(dur)),
                                    "dur_p90": float(np.quantile(dur, 0.9)), "dur_max": float(dur.max()),
                                    "start_p90": float(np.quantile(start, 0.9)), "end_p50": float(np.median(end)),
                                    "visits_p50": float(np.median(vis)), "visits_max": float(vis.max()),
                                    "pairs_p50": float(np.median(prs)), "pairs_max": float(prs.max()),
                                    "slow_wg": [[int(i), float(dur[i]), float(vis[i]), float(prs[i])] for i in slow],
                                    "corr_dur_visits": float(np.corrcoef(dur, vis)[0, 1]),
                                    "corr_dur_pairs": float(np.corrcoef(dur, prs)[0, 1])}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 3, sys.argv[2] if len(sys.argv) > 2 else "around",
         "batch" in sys.argv[3:])
