"""Secondary measurements for BASELINE.json configs other than the headline (bench.py = config 2).

  python tools/bench_configs.py [--only c1,c2opt,c3,c4,c4loop,c5,fit]      (one GPU; prints one JSON line per case)

c1     config 1: banana stored GPIS (N = 361), 64 candidates, Allegro and Leap — closure evals/s
       (launch-bound at this size) next to the oracle on the host cores.
c1opt  config 1 size through the fused optimise loop, eager vs hipGraph replay.
c2opt  config 2 with the optimiser: closure + fused Adam/best-iterate/clamp step, iterations/s.
c3     config 3 objects (stored states, box fit, dummy for realsense), 4096 candidates each — closure
       evals/s per object on one GPU (one object per GPU on a node).
c4     config 4 primitives: iiwa7_allegro FK (23 DOF, 4 tips) fwd+bwd for 16 384 candidates and the
       TorchSDF kernel on the banana mesh (16 384 faces) for the 3 SDF calls of an SDF/Kin-mode iteration
       (tips vs deflated mesh, tips vs mesh, targets vs mesh: 3 × 65 536 points) + SDF backward.
c4loop config 4 loops: prob closure on the iiwa7_allegro chain (23 DOF) with the collision term fused
       (collision=True), 16 384 candidates, N = 2000 GPIS; and the SDF/Kin-mode optimiser
       (KinGraspOptimizer: FK + 3 TorchSDF calls on the banana mesh + force_eq) at 16 384 candidates.
c5     config 5: annealing outer loop (compliancedex_amd.anneal) over 65 536 candidates on one GPU,
       3 outer steps × 30 fused inner iterations, N = 2000 GPIS.
fit    §8f row 2: on-device GPIS fit (R, E11) + factor (Cholesky, E11⁻¹, α) for N = 361 / 1000 / 2000,
       next to torch-CPU fit + inverse (the work the reference does per object) on the host cores.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def timed(fn, reps, warm=2):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def make_opt(hand, palm, dev, iters=1):
    from compliancedex_amd import ProbabilisticGraspOptimizer
    from compliancedex_amd.urdf import load_robot
    cfg = load_robot(hand)["config"]
    return ProbabilisticGraspOptimizer(hand, cfg["ee_link_name"], cfg["ee_link_offset"], palm_offset=palm,
                                       ref_q=cfg["ref_q"], optimize_target=True, optimize_palm=True, device=dev,
                                       num_iters=iters), cfg


def closure_case(hand, gpis, E, dev, center=None, reps=20):
    from compliancedex_amd.workloads import prob_inputs
    opt, cfg = make_opt(hand, np.zeros((E, 6)), dev)
    q, comp, target, palm = prob_inputs(cfg["ref_q"], E, seed=5, spread=True, center=center)
    opt.palm_offset = torch.from_numpy(palm).to(dev)
    t = [torch.from_numpy(a).to(dev).requires_grad_(True) for a in (q, comp, target, palm[:, :3], palm[:, 3:])]

    def step():
        for x in t:
            x.grad = None
        opt.closure(*t, 1, gpis, E)
    sec = timed(step, reps)
    return sec, int((~torch.isfinite(opt.total_loss)).sum())


def case_c1(dev):
    from compliancedex_amd.urdf import load_robot
    from compliancedex_amd.workloads import prob_inputs, stored_gpis
    from oracle.cdx_oracle import OracleChain, OracleGPIS, OracleProblem, closure_with_grads
    g = stored_gpis("banana", dev)
    for hand in ("allegro", "leap"):
        E = 64
        sec, nan = closure_case(hand, g, E, dev, reps=50)
        cfg = load_robot(hand)["config"]
        prob = OracleProblem(OracleChain(load_robot(hand)["bodies"]), cfg["ee_link_name"], cfg["ee_link_offset"],
                             cfg["ref_q"], OracleGPIS.from_npz(os.path.join(REPO, "compliancedex_amd", "data",
                                                                           "gpis_states", "banana_state.npz")))
        q, comp, target, palm = prob_inputs(cfg["ref_q"], E, seed=5, spread=True)
        kn = np.random.default_rng(1).random((3 * E, 3, 3))
        ts = []
        for _ in range(6):
            t0 = time.perf_counter()
            closure_with_grads(prob, q, comp, target, palm, kn)
            ts.append(time.perf_counter() - t0)
        cpu = float(np.median(ts[1:]))
        print(json.dumps({"case": f"config1_{hand}", "E": E, "n_inducing": 361, "gpu_ms_per_closure": sec * 1e3,
                          "gpu_evals_per_s": E / sec, "cpu_oracle_evals_per_s": E / cpu,
                          "cpu_threads": torch.get_num_threads(), "nan_candidates": nan}), flush=True)


def case_c1opt(dev):
    """Config 1 size through the fused optimise loop: eager launches vs one captured hipGraph."""
    from compliancedex_amd.workloads import prob_inputs, stored_gpis
    g = stored_gpis("banana", dev)
    E, iters = 64, 30
    for hand in ("allegro", "leap"):
        opt, cfg = make_opt(hand, np.zeros((E, 6)), dev, iters)
        q, comp, target, palm = prob_inputs(cfg["ref_q"], E, seed=6, spread=True)
        opt.palm_offset = torch.from_numpy(palm).to(dev)
        args = [torch.from_numpy(a).to(dev) for a in (q, target, comp)]
        for graph in (False, True):
            sec = timed(lambda: opt.optimize(*args, 1, g, verbose=False, graph=graph), 5, warm=2)
            print(json.dumps({"case": "config1_optimize", "hand": hand, "graph": graph, "E": E, "iterations": iters,
                              "ms_per_iteration": sec / iters * 1e3, "evals_per_s": E * iters / sec}), flush=True)


def case_c2opt(dev):
    from compliancedex_amd.workloads import prob_inputs, synthetic_banana_gpis
    g = synthetic_banana_gpis(2000, dev)
    E, iters = 4096, 30
    opt, cfg = make_opt("allegro", np.zeros((E, 6)), dev, iters)
    q, comp, target, palm = prob_inputs(cfg["ref_q"], E, seed=6, spread=True)
    opt.palm_offset = torch.from_numpy(palm).to(dev)
    args = [torch.from_numpy(a).to(dev) for a in (q, target, comp)]
    for fused, graph in ((True, False), (True, True), (False, False)):
        sec = timed(lambda: opt.optimize(*args, 1, g, verbose=False, fused=fused, graph=graph), 2, warm=1)
        print(json.dumps({"case": "config2_optimize", "fused_step": fused, "graph": graph, "E": E,
                          "iterations": iters, "ms_per_iteration": sec / iters * 1e3,
                          "evals_per_s": E * iters / sec}), flush=True)


def case_c3(dev):
    from compliancedex_amd.workloads import CONFIG3_OBJECTS, config3_gpis
    for r in range(len(CONFIG3_OBJECTS)):
        name, g = config3_gpis(r, dev)
        X1, y1 = g.X1.cpu().numpy(), g.y1.cpu().numpy().reshape(-1)
        surf = X1[np.abs(y1 - y1.min() if name == "box" else y1 - np.median(y1)) < 1e-9]
        surf = surf if len(surf) else X1
        center = 0.5 * (surf.min(0) + surf.max(0))
        sec, nan = closure_case("allegro", g, 4096, dev, center=center, reps=10)
        print(json.dumps({"case": "config3_object", "object": name, "n_inducing": int(len(X1)), "E": 4096,
                          "ms_per_closure": sec * 1e3, "evals_per_s": 4096 / sec, "nan_candidates": nan}), flush=True)


def case_c4(dev):
    from compliancedex_amd import DifferentiableRobotModel, compute_sdf
    from compliancedex_amd.urdf import load_robot
    E = 16384
    m = DifferentiableRobotModel("iiwa7_allegro", device=dev)
    links = load_robot("iiwa7_allegro")["config"]["ee_link_name"]
    q = (0.3 * torch.randn(E, m._n_dofs, device=dev)).requires_grad_(True)
    off = [[0.0, -0.04, 0.015]] * 4

    def fk():
        q.grad = None
        pos, _ = m.compute_forward_kinematics(q, links, offsets=off)
        pos.sum().backward()
    fk_s = timed(fk, 20)
    faces = torch.from_numpy(np.load(os.path.join(REPO, "compliancedex_amd", "data", "meshes",
                                                  "banana_faces.npy"))).to(dev)
    lo, hi = faces.reshape(-1, 3).min(0)[0], faces.reshape(-1, 3).max(0)[0]
    pts = [(lo - 0.02 + (hi - lo + 0.04) * torch.rand(4 * E, 3, device=dev)).requires_grad_(True) for _ in range(3)]
    deflated = faces * 0.9

    def sdf():
        outs = [compute_sdf(pts[0], deflated), compute_sdf(pts[1], faces), compute_sdf(pts[2], faces)]
        sum(o[0].sum() for o in outs).backward()
    sdf_s = timed(sdf, 5, warm=1)
    pairs = 3 * 4 * E * faces.shape[0]
    # forward alone (HIP events on the stream: the whole cdx_sdf_forward launch sequence) and the
    # culled kernel's work counters (cdx_sdf_stats): pairs evaluated after culling vs brute force
    import ctypes
    from compliancedex_amd import _native as N
    lib = N.load()
    st = (ctypes.c_uint64 * 3)()
    N.check(lib.cdx_sdf_stats(1, None, N.stream_ptr(dev)), "cdx_sdf_stats")
    with torch.no_grad():
        for i, f in enumerate((deflated, faces, faces)):
            compute_sdf(pts[i].detach(), f)
    N.check(lib.cdx_sdf_stats(0, st, N.stream_ptr(dev)), "cdx_sdf_stats")
    visits = ctypes.c_uint64(0)
    N.check(lib.cdx_sdf_chunk_visits(ctypes.byref(visits), N.stream_ptr(dev)), "cdx_sdf_chunk_visits")
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    reps = 10
    with torch.no_grad():
        for i, f in enumerate((deflated, faces, faces)):
            compute_sdf(pts[i].detach(), f)
        ev[0].record()
        for _ in range(reps):
            for i, f in enumerate((deflated, faces, faces)):
                compute_sdf(pts[i].detach(), f)
        ev[1].record()
    torch.cuda.synchronize()
    fwd_ms = ev[0].elapsed_time(ev[1]) / reps
    evaluated, brute_exact, n_pts = int(st[0]), int(st[1]), int(st[2])
    flops_pair = 46  # f32 flops of face_dist2 on its usual branch (cdx_sdf.h; 3 IEEE divisions counted as 1 each)
    achieved = (evaluated + brute_exact) * flops_pair / (fwd_ms * 1e-3) / 1e12
    print(json.dumps({"case": "config4_primitives", "E": E, "fk_fwd_bwd_ms": fk_s * 1e3,
                      "fk_evals_per_s": E / fk_s, "sdf_3calls_fwd_bwd_ms": sdf_s * 1e3,
                      "sdf_point_face_pairs_per_s": pairs / sdf_s, "faces": int(faces.shape[0]),
                      "sdf_evals_per_s": E / sdf_s,
                      "roofline_sdf": {"bound": "valu", "kernel": "sdf_tree_kernel, one-shot compute_sdf (+ per-call Morton mesh build and point sort)",
                                       "fwd_3calls_ms": fwd_ms, "points": n_pts, "brute_force_pairs": pairs,
                                       "pairs_evaluated": evaluated, "pairs_exact_path": brute_exact,
                                       "chunk_visits_per_wave": int(visits.value) / max(1, 4 * ((n_pts + 63) // 64)),
                                       "chunks": (int(faces.shape[0]) + 31) // 32,
                                       "evaluated_over_brute_force": (evaluated + brute_exact) / pairs,
                                       "flops_per_pair": flops_pair, "achieved": achieved, "peak": 157.3,
                                       "unit": "TFLOP/s (f32 vector)", "frac": achieved / 157.3,
                                       "note": "achieved counts only the evaluated pairs' face_dist2 flops over the "
                                               "whole forward (sorts, culling tests, winner recompute included)"}}),
          flush=True)


def case_c4loop(dev):
    from compliancedex_amd import KinGraspOptimizer, ProbabilisticGraspOptimizer, TriangleMesh
    from compliancedex_amd.urdf import load_robot
    from compliancedex_amd.workloads import prob_inputs, synthetic_banana_gpis
    E = 16384
    links = load_robot("iiwa7_allegro")["config"]["ee_link_name"]
    D = 23
    ref_q = [0.0] * D
    offs = [[0.0, -0.04, 0.015]] * 3 + [[0.0, -0.05, -0.015]]
    g = synthetic_banana_gpis(2000, dev)
    q, comp, target, _ = prob_inputs(ref_q, E, seed=8, spread=True)
    q = 0.05 * np.random.default_rng(9).standard_normal((E, D))
    # the "palm" pose is the arm base here: place it so the fingertips at q = 0 surround the banana
    from compliancedex_amd import DifferentiableRobotModel
    tips0 = DifferentiableRobotModel("iiwa7_allegro", device=dev).compute_forward_kinematics(
        torch.zeros(1, D, device=dev), links, offsets=offs)[0].view(4, 3).double().mean(0).cpu().numpy()
    center = np.load(os.path.join(REPO, "compliancedex_amd", "data", "banana_center.npy"))
    rng = np.random.default_rng(8)
    palm = np.concatenate([center - tips0 + 0.005 * rng.standard_normal((E, 3)), 0.02 * rng.standard_normal((E, 3))], 1)
    pairs = [[0, 1], [0, 2], [0, 3], [1, 2], [1, 3], [2, 3]]
    opt = ProbabilisticGraspOptimizer("iiwa7_allegro", links, offs, palm_offset=palm, ref_q=ref_q,
                                      optimize_target=True, optimize_palm=True, device=dev, anchor_link_names=links,
                                      anchor_link_offsets=offs, collision_pairs=pairs, collision=True)
    t = [torch.from_numpy(a).to(dev).requires_grad_(True) for a in (q, comp, target, palm[:, :3], palm[:, 3:])]

    def step():
        for x in t:
            x.grad = None
        opt.closure(*t, 1, g, E)
    sec = timed(step, 10)
    print(json.dumps({"case": "config4_closure_iiwa7_collision", "E": E, "n_dofs": D, "n_inducing": 2000,
                      "ms_per_closure": sec * 1e3, "evals_per_s": E / sec,
                      "nan_candidates": int((~torch.isfinite(opt.total_loss)).sum())}), flush=True)
    mesh = TriangleMesh.from_npz(os.path.join(REPO, "compliancedex_amd", "data", "meshes", "banana_mesh.npz"))
    iters = 20  # amortises the per-call setup (mesh upload, face-chunk culling structure)
    kin = KinGraspOptimizer("iiwa7_allegro", links, offs, palm_offset=[0.0, 0.0, 0.0], num_iters=iters,
                            optimize_target=True, ref_q=ref_q)
    qf = (0.3 * torch.randn(E, D, device=dev)).float()
    tg = torch.from_numpy(target).to(dev).float()
    cp = torch.from_numpy(comp).to(dev).float()

    kin.loop_events = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    loop_ms = []

    def loop():
        kin.optimize(qf, tg, cp, 1, TriangleMesh(mesh.vertices, mesh.triangles), verbose=False)
        torch.cuda.synchronize()
        loop_ms.append(kin.loop_events[0].elapsed_time(kin.loop_events[1]))
    sec = timed(loop, 3, warm=1)
    it_ms = min(loop_ms[1:]) / iters
    print(json.dumps({"case": "config4_kin_sdf_loop", "E": E, "iterations": iters, "faces": int(len(mesh.triangles)),
                      "ms_per_iteration_whole_call": sec / iters * 1e3, "ms_per_iteration_loop": it_ms,
                      "per_call_setup_ms": sec * 1e3 - it_ms * iters, "evals_per_s_loop": E / it_ms * 1e3,
                      "note": "whole call = per-call setup (mesh upload, two prepared meshes, state) + the loop; the "
                              "reference's default is 1000 iterations per call"}), flush=True)


def case_c4kin(dev):
    """The SDF/Kin-mode loop alone (for a per-kernel rocprof split of one iteration)."""
    from compliancedex_amd import KinGraspOptimizer, TriangleMesh
    from compliancedex_amd.urdf import load_robot
    from compliancedex_amd.workloads import prob_inputs
    E, D, iters = 16384, 23, int(os.environ.get("CDX_C4KIN_ITERS", "20"))
    links = load_robot("iiwa7_allegro")["config"]["ee_link_name"]
    offs = [[0.0, -0.04, 0.015]] * 3 + [[0.0, -0.05, -0.015]]
    _, comp, target, _ = prob_inputs([0.0] * D, E, seed=8, spread=True)
    mesh = TriangleMesh.from_npz(os.path.join(REPO, "compliancedex_amd", "data", "meshes", "banana_mesh.npz"))
    kin = KinGraspOptimizer("iiwa7_allegro", links, offs, palm_offset=[0.0, 0.0, 0.0], num_iters=iters,
                            optimize_target=True, ref_q=[0.0] * D)
    qf = (0.3 * torch.randn(E, D, device=dev)).float()
    tg = torch.from_numpy(target).to(dev).float()
    cp = torch.from_numpy(comp).to(dev).float()

    def loop():
        kin.optimize(qf, tg, cp, 1, TriangleMesh(mesh.vertices, mesh.triangles), verbose=False)
    sec = timed(loop, 3, warm=1)
    # the culled forward's work counters over one more loop (after the timing): pairs evaluated per call
    import ctypes
    from compliancedex_amd import _native as N
    lib = N.load()
    st = (ctypes.c_uint64 * 3)()
    visits = ctypes.c_uint64(0)
    N.check(lib.cdx_sdf_stats(1, None, N.stream_ptr(dev)), "cdx_sdf_stats")
    N.check(lib.cdx_sdf_chunk_visits(ctypes.byref(visits), N.stream_ptr(dev)), "cdx_sdf_chunk_visits")
    loop()
    N.check(lib.cdx_sdf_stats(0, st, N.stream_ptr(dev)), "cdx_sdf_stats")
    N.check(lib.cdx_sdf_chunk_visits(ctypes.byref(visits), N.stream_ptr(dev)), "cdx_sdf_chunk_visits")
    calls = max(1, int(st[2]) // (4 * E))
    print(json.dumps({"case": "config4_kin_sdf_loop", "E": E, "iterations": iters, "faces": int(len(mesh.triangles)),
                      "ms_per_iteration": sec / iters * 1e3, "evals_per_s": E * iters / sec,
                      "sdf_calls": calls, "pairs_evaluated_per_call": int(st[0]) / calls,
                      "pairs_exact_path_per_call": int(st[1]) / calls,
                      "brute_force_pairs_per_call": 4 * E * len(mesh.triangles),
                      "chunk_visits_per_point_group_wave": int(visits.value) / max(1, 4 * (int(st[2]) // 64))}),
          flush=True)


def case_c5(dev):
    from compliancedex_amd import PregraspAnnealer, ProbabilisticGraspOptimizer
    from compliancedex_amd.urdf import load_robot
    from compliancedex_amd.workloads import prob_inputs, synthetic_banana_gpis
    E, inner, outer = 65536, 30, 3
    cfg = load_robot("allegro")["config"]
    g = synthetic_banana_gpis(2000, dev)
    q, comp, target, palm = prob_inputs(cfg["ref_q"], E, seed=9, spread=True)
    opt = ProbabilisticGraspOptimizer("allegro", cfg["ee_link_name"], cfg["ee_link_offset"], palm_offset=palm,
                                      ref_q=cfg["ref_q"], optimize_target=True, optimize_palm=True, device=dev,
                                      num_iters=inner)
    t = [torch.from_numpy(a).to(dev) for a in (q, target, comp, palm)]
    ann = PregraspAnnealer(opt, g, seed=1)
    res = {}

    def run():
        res["best"] = ann.run(*t, outer_steps=outer)
    sec = timed(run, 1, warm=1)
    best = res["best"]
    surv = int((best["margin"] > 0).all(1).sum())
    print(json.dumps({"case": "config5_anneal", "E": E, "inner_iterations": inner, "outer_steps": outer,
                      "seconds": sec, "evals_per_s": E * inner * outer / sec,
                      "finite_best": int(torch.isfinite(best["loss"]).sum()), "surviving_grasps": surv,
                      "mean_accepts": float(best["accepted"].double().mean())}), flush=True)


def case_fit(dev):
    from compliancedex_amd import GPIS
    from compliancedex_amd.workloads import synthetic_banana_arrays
    from oracle.cdx_oracle import OracleGPIS
    for n in (361, 1000, 2000):
        X1, y, noise = synthetic_banana_arrays(n)
        Xd, yd, nd = (torch.from_numpy(a).to(dev) for a in (X1, y, noise))
        g = GPIS(0.08, 1.0)

        def fit():
            g.fit(Xd, yd, noise=nd)
            g.native_state()
        sec = timed(fit, 5)
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            o = OracleGPIS.fit(X1, y, noise, bias=1.0)
            torch.linalg.inv(o.E11)
            ts.append(time.perf_counter() - t0)
        print(json.dumps({"case": "fit_factor", "n_inducing": n, "gpu_ms": sec * 1e3,
                          "cpu_torch_fit_inverse_ms": float(np.median(ts)) * 1e3,
                          "cpu_threads": torch.get_num_threads()}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="c1,c2opt,c3,c4,c4loop,c5,fit")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    for c in args.only.split(","):
        globals()[f"case_{c}"](dev)


if __name__ == "__main__":
    main()
