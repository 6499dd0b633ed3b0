"""Benchmark: candidate-grasp cost+grad evals/sec (BASELINE.json metric), configs 2 and 3.

One step = one prob-mode closure (forward + backward, optimize_pregrasp.py:741-769) over
E candidates per GPU with the Allegro hand — the whole hot path (FK → GPIS mean/normal/std →
cost + analytic backward) through the C ABI.

Workload = config 3 as north_star states it, which at one GPU is config 2: rank r owns object r
of workloads.CONFIG3_OBJECTS (banana, mug, mug2, hammer, lego, coffeebottle, box, realsense
stand-in), each an N = 2000 GPIS fitted with the config-2 recipe (rank 0's banana IS config 2's
synthetic state), E = 4096 candidates around the object.  No collective inside the steps; the
timed region ends with the path's one exchange step: every rank packs its surviving grasps (all
four margins > 0) into fixed-capacity records and one all_gather (RCCL over xGMI) gives every
rank all objects' survivors (distributed.py).  Per-GPU work is fixed as N grows
(weak scaling).

  python bench.py [--gpus N --steps K --warmup W --E 4096 --n-inducing 2000]
  N > 1: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

FP64_MFMA_PEAK_TFLOPS = 78.6  # gfx950 vendor spec; MI355X_MICROARCH.md has no f64 row
F16_MFMA_PEAK_TFLOPS = 2500.0  # dense fp16/bf16 MFMA (MI355X_MICROARCH.md § Matrix cores)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    # the GPU clock ramps over the first ~10 closures (1.92 → 1.77 ms, tools/clock_ramp.py): warm past it
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--E", type=int, default=4096, help="candidates per GPU")
    ap.add_argument("--n-inducing", type=int, default=2000)
    ap.add_argument("--hand", default="allegro")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-E", type=int, default=256)
    ap.add_argument("--backend", default="nccl", help="nccl (= RCCL, default) or gloo (rehearsal on one GPU)")
    ap.add_argument("--no-config4", action="store_true", help="skip the config-4 SDF/Kin block (N = 1)")
    ap.add_argument("--config4-iters", type=int, default=1000)  # (the reference's Kin loop default: 1000 per call)
    return ap.parse_args()


def cpu_quota():
    """CPUs this process may use: the cgroup quota (cpu.max) if set, else the affinity mask."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            return max(1, int(int(q) / int(p)))
    except (OSError, ValueError):
        pass
    return len(os.sched_getaffinity(0))


def cpu_baseline(args, ref_q, cfg):
    """Oracle (CPU restatement of the reference path) on a bounded sample of the same workload,
    with torch's intra-op threads = the CPUs this job may use (the GPU box allots 16 per GPU:
    os.cpu_count() reports the whole machine, whose other cores run other jobs)."""
    import numpy as np
    import torch

    from compliancedex_amd.urdf import load_robot
    from compliancedex_amd.workloads import prob_inputs, synthetic_banana_arrays
    from oracle.cdx_oracle import OracleChain, OracleGPIS, OracleProblem, closure_with_grads

    X1, y, noise = synthetic_banana_arrays(args.n_inducing)
    prob = OracleProblem(OracleChain(load_robot(args.hand)["bodies"]), cfg["ee_link_name"], cfg["ee_link_offset"],
                         ref_q, OracleGPIS.fit(X1, y, noise, bias=1.0))
    E = args.cpu_E
    threads = cpu_quota()
    torch.set_num_threads(threads)
    q, comp, target, palm = prob_inputs(ref_q, E, seed=99, spread=True)
    kn = np.random.default_rng(98).random((3 * E, 3, 3))
    times = []
    for i in range(4):
        t0 = time.perf_counter()
        closure_with_grads(prob, q, comp, target, palm, kn)
        times.append(time.perf_counter() - t0)
    med = statistics.median(times[1:])
    return {"value": E / med, "unit": "evals/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"oracle/cdx_oracle.py closure (reference algorithm incl. per-call LU solve and M×M "
                      f"posterior), E={E} candidates, N={args.n_inducing} GPIS, {args.hand}; median of 3 after "
                      f"1 warm-up; torch threads = the job's CPU quota ({threads}); host "
                      f"os.cpu_count()={os.cpu_count()} (whole machine)"}


def hbm_traffic(E, n, key="gpis_var_bytes_per_launch"):
    """Per-launch HBM bytes of a GEMM kernel, measured by rocprofv3 PMC counters on the same
    workload: profiles/pmc_traffic.json (tools/pmc_summary.py writes it from the newest
    profiles/TAG_pmc.json; it is the one file of profiles/ shipped to the GPU box), else the newest
    matching profiles/*_pmc.json.  (gfx950-corrected: (2·FETCH_SIZE + WRITE_SIZE)·1 KiB.)"""
    import glob
    cands = [os.path.join(REPO, "profiles", "pmc_traffic.json")] + \
        sorted(glob.glob(os.path.join(REPO, "profiles", "*_pmc.json")), reverse=True)
    for p in cands:
        try:
            d = json.load(open(p))
        except Exception:
            continue
        if d.get("E") == E and d.get("n_inducing") == n and key in d:
            return d[key], d.get("source", os.path.relpath(p, REPO))
    return None, None


def traffic_block(E, n, key, algorithmic):
    """roofline.traffic (PMC bytes per launch), the algorithmic bytes beside it and their ratio."""
    t, src = hbm_traffic(E, n, key)
    return {"traffic": t, "traffic_source": src, "algorithmic_bytes": algorithmic,
            "traffic_over_algorithmic": (t / algorithmic) if (t and algorithmic) else None}


CONFIG3 = ["banana", "mug", "mug2", "hammer", "lego", "coffeebottle", "box", "realsense"]
F32_VALU_PEAK_TFLOPS = 157.3  # gfx950 f32 vector (MI355X_MICROARCH.md)
SDF_FLOPS_PER_PAIR = 46       # face_dist2's usual branch, 3 IEEE divisions counted as 1 flop each (cdx_sdf.h)


def config4_kin(args, dev):
    """Config 4's SDF leg (BASELINE configs[3]: iiwa7_allegro arm + hand, TorchSDF on): the fused KinGraspOptimizer
    loop (optimize_pregrasp.py:183-223) at E = 16 384 candidates on the 16 384-face banana — per iteration three
    TorchSDF queries on prepared meshes (3 × 65 536 points) and cdx_kin_iteration (cost, backward and step) — timed over
    ``--config4-iters`` iterations after a warm-up call (HIP events on the loop's stream), then the three queries
    of one iteration alone (the TorchSDF forward) and the culled kernel's work counters."""
    import copy
    import ctypes

    import torch

    from compliancedex_amd import KinGraspOptimizer
    from compliancedex_amd import _native as N
    from compliancedex_amd.workloads import banana_mesh, config4_kin_inputs

    lib = N.load()
    E, iters = 16384, args.config4_iters
    links, offs, palm, q, target, comp = config4_kin_inputs(E, device=dev)
    kin = KinGraspOptimizer("iiwa7_allegro", links, offs, palm_offset=palm.tolist(), num_iters=iters,
                            optimize_target=True, ref_q=[0.0] * 23, device=dev)
    x = [torch.from_numpy(a).to(dev) for a in (q, target, comp)]
    mesh = banana_mesh()
    kin.optimize(*x, 1, copy.deepcopy(mesh), verbose=False)  # warm-up: prepares, allocator, clocks
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    # the timed region: the iterations (the two meshes are prepared once per optimize call, before it)
    kin.loop_events = ev[:2]
    mesh_c = copy.deepcopy(mesh)
    torch.cuda.synchronize()
    t_call = time.perf_counter()
    res = kin.optimize(*x, 1, mesh_c, verbose=False)
    torch.cuda.synchronize()
    t_call = time.perf_counter() - t_call
    kin.loop_events = None
    ms_iter = ev[0].elapsed_time(ev[1]) / iters
    # the reference's non-finite case (:212-213): candidates whose last-iteration loss is not finite, and fingertips
    # with a non-finite coordinate after the last step
    nonfinite = int((~torch.isfinite(kin.last_loss)).sum())
    nonfinite_tips = int((~torch.isfinite(kin.last_tips)).any(dim=1).sum())
    # the same loop over 20 iterations (before any candidate diverges: DESIGN §5b), timed the same way
    kin20 = KinGraspOptimizer("iiwa7_allegro", links, offs, palm_offset=palm.tolist(), num_iters=20,
                              optimize_target=True, ref_q=[0.0] * 23, device=dev)
    kin20.loop_events = ev[2:]
    kin20.optimize(*x, 1, copy.deepcopy(mesh), verbose=False)
    torch.cuda.synchronize()
    ms_iter20 = ev[2].elapsed_time(ev[3]) / 20
    nonfinite20 = int((~torch.isfinite(kin20.last_loss)).sum())
    # the TorchSDF forward of one iteration alone (the loop's three queries on its final fingertips / targets)
    from compliancedex_amd import PreparedMesh
    from compliancedex_amd.optimizers import _face_vertices
    from compliancedex_amd.torchsdf import QueryWorkspace
    m = copy.deepcopy(mesh)
    faces = _face_vertices(m, dev)
    m.scale(0.9, center=[0, 0, 0])
    full = PreparedMesh(faces)
    meshes = (PreparedMesh(_face_vertices(m, dev)), full, full)
    ws_t, ws_g = QueryWorkspace(), QueryWorkspace()
    wss = (ws_t, ws_t, ws_g)
    from compliancedex_amd import DifferentiableRobotModel
    tips = (DifferentiableRobotModel("iiwa7_allegro", device=dev).compute_forward_kinematics(
        res[0].detach(), links, offsets=offs)[0].view(-1, 3) + torch.from_numpy(palm).to(dev)).contiguous()
    pts = (tips, tips, res[2].detach().reshape(-1, 3).contiguous())
    from compliancedex_amd.torchsdf import BatchSchedule, query_batch
    sched = BatchSchedule()
    P = pts[0].shape[0]
    outs = [(torch.empty(P, device=dev), torch.empty(P, dtype=torch.int32, device=dev), torch.empty(P, 3, device=dev),
             torch.empty(P, 3, device=dev)) for _ in range(3)]

    def three():
        """The loop's pattern on a re-sorting iteration (optimizers._FusedLoop.queries): both point sets sorted, then
        the three queries in one launch (cdx_sdf_query_batch) with the loop's schedule (heaviest groups first)."""
        ws_t.sort(tips)
        ws_g.sort(pts[2])
        query_batch([(meshes[k], pts[k], wss[k], outs[k]) for k in range(3)], schedule=sched)
    three()
    st = (ctypes.c_uint64 * 3)()
    visits = ctypes.c_uint64(0)
    N.check(lib.cdx_sdf_stats(1, None, N.stream_ptr(dev)), "cdx_sdf_stats")
    three()
    N.check(lib.cdx_sdf_stats(0, st, N.stream_ptr(dev)), "cdx_sdf_stats")
    N.check(lib.cdx_sdf_chunk_visits(ctypes.byref(visits), N.stream_ptr(dev)), "cdx_sdf_chunk_visits")
    reps = 10
    ev[2].record()
    for _ in range(reps):
        three()
    ev[3].record()
    torch.cuda.synchronize()
    fwd_ms = ev[2].elapsed_time(ev[3]) / reps
    n_pts, F = int(st[2]), int(faces.shape[0])
    brute = n_pts * F
    evaluated = int(st[0]) + int(st[1])
    achieved = evaluated * SDF_FLOPS_PER_PAIR / (fwd_ms * 1e-3) / 1e12
    brute_eq = brute * SDF_FLOPS_PER_PAIR / (fwd_ms * 1e-3) / 1e12
    return {"workload": "config 4: KinGraspOptimizer (fused) on iiwa7_allegro (23 DOF, chain depth 13), "
                        f"E={E} candidates, 16 384-face banana mesh, optimize_target, 3 TorchSDF queries per iteration",
            "iterations": iters, "ms_per_iteration": ms_iter, "evals_per_s": E / (ms_iter * 1e-3),
            "nonfinite_candidates": nonfinite, "nonfinite_fingertips": nonfinite_tips,
            "call_ms": t_call * 1e3, "setup_ms": t_call * 1e3 - ms_iter * iters,
            "ms_per_iteration_20": ms_iter20, "nonfinite_candidates_20": nonfinite20,
            "timing_note": "ms_per_iteration: HIP events around the iterations of one optimize call (device Kabsch "
                           "noise); call_ms: host wall time of that whole call (setup_ms = call_ms − the iterations: "
                           "the two meshes' preparation with their host k-d builds and uploads, the loop state, one "
                           "host wait); ms_per_iteration_20: a 20-iteration call timed the same way",
            "launches_per_iteration": "3 TorchSDF queries in one launch (sdf_tree_batch_kernel, heaviest point groups of "
                                      "the last iteration first, + its one-workgroup schedule kernel; the fingertips' and "
                                      "the targets' Morton order — bbox partials, keys, an 18-bit radix sort — every 16th "
                                      "iteration) + cdx_kin_iteration (cost, backward, best iterate, Adam, next "
                                      "fingertips: one launch)",
            "roofline_sdf": {"bound": "valu", "kernel": "sdf_tree_kernel (+ per-query bbox, Morton keys, radix sort)",
                             "fwd_3calls_ms": fwd_ms, "fwd_pattern": "both point sets sorted, the three queries in one launch (the "
                                                               "loop's iterations re-sort every 16th)", "points": n_pts, "faces": F, "brute_force_pairs": brute,
                             "pairs_evaluated": int(st[0]), "pairs_exact_path": int(st[1]),
                             "pairs_per_point": int(st[0]) / max(1, n_pts),
                             "chunk_visits_per_wave": int(visits.value) / max(1, (n_pts + 63) // 64),
                             "evaluated_over_brute_force": evaluated / brute,
                             "flops_per_pair": SDF_FLOPS_PER_PAIR, "achieved": achieved, "peak": F32_VALU_PEAK_TFLOPS,
                             "unit": "TFLOP/s (f32 vector)", "frac": achieved / F32_VALU_PEAK_TFLOPS,
                             "brute_force_equivalent": brute_eq,
                             "note": "achieved counts only the evaluated pairs' face_dist2 flops over the three "
                                     "queries' whole forward (sorts and culling tests included), so it falls as the "
                                     "culling improves; brute_force_equivalent = the reference's brute-force pair "
                                     "flops (P·F·46) over the same time"}}


def config4_closure(args, dev, gpis):
    """Config 4 as BASELINE states it (configs[3]: "AllegroHand on kuka_allegro arm FK chain + TorchSDF self-collision
    enabled, 16 384 candidates, bf16 GPIS kernel-matrix on MFMA"): the prob-mode closure (optimize_pregrasp.py:741-769)
    with compute_collision_loss fused in (:671-701; the reference leaves the call commented out at :765) on iiwa7_allegro
    (23 DOF, chain depth 13), E = 16 384 candidates around config 2's N = 2000 banana GPIS.  The GPIS kernel-matrix
    product's low-precision MFMA leg is the fp16 2-slice screen (gpis_screen_kernel); every value that reaches the loss
    comes from the fp64 MFMA passes.  Timed over 10 closures after 5 warm-up (HIP events on the closure's
    stream), then a 5-closure all-stage pass for the three GEMM kernels' rooflines."""
    import ctypes

    import numpy as np
    import torch

    from compliancedex_amd import DifferentiableRobotModel, ProbabilisticGraspOptimizer
    from compliancedex_amd import _native as N
    from compliancedex_amd.urdf import load_robot
    from compliancedex_amd.workloads import CONFIG4_OFFSETS, prob_inputs

    E, D = 16384, 23
    links = load_robot("iiwa7_allegro")["config"]["ee_link_name"]
    ref_q = [0.0] * D
    _, comp, target, _ = prob_inputs(ref_q, E, seed=8, spread=True)
    rng = np.random.default_rng(9)
    q = 0.05 * rng.standard_normal((E, D))
    # the "palm" pose is the arm base: placed so the fingertips at q = 0 surround the banana
    tips0 = DifferentiableRobotModel("iiwa7_allegro", device=dev).compute_forward_kinematics(
        torch.zeros(1, D, device=dev), links, offsets=CONFIG4_OFFSETS)[0].view(4, 3).double().mean(0).cpu().numpy()
    center = np.load(os.path.join(REPO, "compliancedex_amd", "data", "banana_center.npy"))
    palm = np.concatenate([center - tips0 + 0.005 * rng.standard_normal((E, 3)), 0.02 * rng.standard_normal((E, 3))], 1)
    pairs = [[0, 1], [0, 2], [0, 3], [1, 2], [1, 3], [2, 3]]
    opt = ProbabilisticGraspOptimizer("iiwa7_allegro", links, CONFIG4_OFFSETS, palm_offset=palm, ref_q=ref_q,
                                      optimize_target=True, optimize_palm=True, device=dev, anchor_link_names=links,
                                      anchor_link_offsets=CONFIG4_OFFSETS, collision_pairs=pairs, collision=True)
    t = [torch.from_numpy(np.ascontiguousarray(a)).to(dev).requires_grad_(True)
         for a in (q, comp, target, palm[:, :3], palm[:, 3:])]

    def step():
        for x in t:
            x.grad = None
        opt.closure(*t, 1, gpis, E)
    for _ in range(5):
        step()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    reps = 10
    torch.cuda.synchronize()
    ev[0].record()
    for _ in range(reps):
        step()
    ev[1].record()
    torch.cuda.synchronize()
    ms = ev[0].elapsed_time(ev[1]) / reps
    lib = N.load()
    msa = (ctypes.c_double * N.PROF_STAGES)()
    cnt = (ctypes.c_int64 * N.PROF_STAGES)()
    N.check(lib.cdx_profile_read(msa, cnt), "cdx_profile_read")  # (clears the main run's counts)
    N.check(lib.cdx_profile_enable((1 << N.PROF_STAGES) - 1), "cdx_profile_enable")
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    N.check(lib.cdx_profile_read(msa, cnt), "cdx_profile_read")
    lib.cdx_profile_enable(0)
    names = ["queries", "gpis_mean", "gpis_std_var", "cost_bwd", "gpis_std_grad", "gpis_screen"]
    stage = {n: (msa[i] / cnt[i] if cnt[i] else None) for i, n in enumerate(names)}
    n_ind = args.n_inducing
    lq = opt.problem(gpis, 1).n_query_levels
    m_std, m_grad = lq * E * 4, lq * E
    scr = opt.screen_stats(gpis, E)
    m_exact = scr["exact_rows"] if scr else m_std
    tri = float(n_ind) * (n_ind + 1)

    def roof(kernel, flops, ms_k, peak, note):
        a = flops / (ms_k * 1e-3) / 1e12 if ms_k else None
        return {"bound": "mfma", "kernel": kernel, "achieved": a, "peak": peak, "unit": "TFLOP/s",
                "frac": (a / peak) if a else None, "flops_per_launch": flops, "ms": ms_k, "note": note}
    out = {"workload": "config 4: prob-mode closure fwd+bwd with compute_collision_loss fused (6 fingertip pairs, anchor "
                       f"and palm floor terms), iiwa7_allegro (23 DOF, chain depth 13), E={E} candidates, N={n_ind} banana "
                       "GPIS (config 2's), 3 pregrasp levels; fp16 2-slice MFMA screen + exact fp64 MFMA passes",
           "ms_per_closure": ms, "evals_per_s": E / (ms * 1e-3), "closures_timed": reps,
           "nan_candidates": int((~torch.isfinite(opt.total_loss)).sum()), "stage_ms": stage,
           "roofline": roof("gpis_std_kernel<VARL> (v_mfma_f64_16x16x4_f64, K*·L⁻ᵀ, screened rows)" if scr else
                            "gpis_std_kernel<VAR> (v_mfma_f64_16x16x4_f64, K*·L⁻ᵀ)", m_exact * tri,
                            stage["gpis_std_var"], FP64_MFMA_PEAK_TFLOPS,
                            f"{m_exact} of {m_std} all-tip rows x N(N+1), exact fp64 whitened form"),
           "roofline_grad": roof("gpis_std_kernel<GRADV> (∇std)", m_grad * tri, stage["gpis_std_grad"],
                                 FP64_MFMA_PEAK_TFLOPS, f"{m_grad} argmax-fingertip queries x N(N+1)"),
           "timing_note": "ms_per_closure: HIP events over 10 closures after 5 warm-up; stage ms (rooflines) from a "
                          "5-closure pass with every stage's events on, after it"}
    if scr:
        out["roofline_screen"] = roof("gpis_screen_kernel (v_mfma_f32_32x32x16_f16, 2-slice fp16 split)",
                                      3 * m_std * tri, stage["gpis_screen"], F16_MFMA_PEAK_TFLOPS,
                                      f"{m_std} all-tip rows x 3 x N(N+1) fp16 MFMA flops")
        out["exact_rows"] = m_exact
    return out


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local = local % max(torch.cuda.device_count(), 1)  # ranks share a GPU only in gloo rehearsals
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.backend)

    from compliancedex_amd import ProbabilisticGraspOptimizer
    from compliancedex_amd import _native as N
    from compliancedex_amd import distributed as D
    from compliancedex_amd.urdf import load_robot
    from compliancedex_amd.workloads import config3_gpis, prob_inputs, surface_center

    cfg = load_robot(args.hand)["config"]
    ref_q = cfg["ref_q"]
    E = args.E
    obj, gpis = config3_gpis(rank, dev, n_total=args.n_inducing)
    center = None if obj == "banana" else surface_center(gpis)  # banana: config 2's mesh centre
    q, comp, target, palm = prob_inputs(ref_q, E, seed=1000 + rank, spread=True, center=center)
    opt = ProbabilisticGraspOptimizer(args.hand, cfg["ee_link_name"], cfg["ee_link_offset"], palm_offset=palm,
                                      ref_q=ref_q, optimize_target=True, optimize_palm=True, device=dev, seed=rank << 32)
    qt = torch.from_numpy(q).to(dev).requires_grad_(True)
    ct = torch.from_numpy(comp).to(dev).requires_grad_(True)
    tt = torch.from_numpy(target).to(dev).requires_grad_(True)
    pp = torch.from_numpy(palm[:, :3]).to(dev).requires_grad_(True)
    po = torch.from_numpy(palm[:, 3:]).to(dev).requires_grad_(True)

    def step():
        qt.grad = ct.grad = tt.grad = pp.grad = po.grad = None
        opt.closure(qt, ct, tt, pp, po, 1, gpis, E)

    def exchange(check_shape=True):
        """Surviving grasps of this rank's object → one all_gather of fixed-capacity records
        (capacity E on every rank; the header keeps the true count).  The buffer shapes are checked
        equal across ranks first (one all_reduce and its host read), as every library caller does."""
        buf = D.pack_survivors(E, rank, rank, 0, opt.total_loss, opt.total_margin, qt.detach(), ct.detach(),
                               tt.detach(), torch.cat([pp, po], 1).detach())
        if world > 1:
            records, bufs = D.all_gather_survivors(buf if args.backend == "nccl" else buf.cpu(), return_buffers=True,
                                                   check_shape=check_shape)
        else:
            records, bufs = D.unpack_records([buf]), [buf]
        return buf, records, bufs

    lib = N.load()
    import ctypes
    # Host-side setup that idles the GPU goes BEFORE the warm-up steps, so the timed steps start at the
    # clock the warm-up reached: the profiling event pool (cdx_profile_enable creates 49 152 events on
    # first use) and the exchange's first run (pack kernels, communicator setup, one host read), here on
    # the parameters with zero losses / margins (no survivors; the same buffer shapes).
    N.check(lib.cdx_profile_enable((1 << N.PROF_STAGES) - 1), "cdx_profile_enable")
    N.check(lib.cdx_profile_enable(0), "cdx_profile_enable")
    opt.total_loss = torch.zeros(E, dtype=torch.float64, device=dev)
    opt.total_margin = torch.zeros(E, ct.shape[1], dtype=torch.float64, device=dev)
    exchange()  # warms the pack kernels and the communicator (RCCL sets up its rings on first use)
    for _ in range(args.warmup):
        step()
    # HIP events only around the two roofline kernels inside the timed region (each event record
    # costs ≈ 5 µs of stream time); the other stages are timed in a separate pass afterwards
    # (each record costs stream time: only the dominant kernel's — the exact-pass refine, whose roofline
    # is the headline — is marked in the timed steps; the screen and ∇std kernels in the pass after)
    PROF_TIMED = int(os.environ.get("CDX_BENCH_PROF_TIMED", str(1 << 2)))  # gpis_std_var (refine)
    N.check(lib.cdx_profile_enable(PROF_TIMED), "cdx_profile_enable")
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # per-step stream times of the first and last 5 timed steps (the clock ramp): events between those
    # steps on the closure's stream — each record costs ≈ 8 µs of stream time (profiles/r04b_ab_*: 1.058
    # vs 1.050 ms per step with one between every step), so only the 12 boundaries are marked
    # (CDX_BENCH_STEP_EVENTS=0 drops them, =all marks every step)
    mode = os.environ.get("CDX_BENCH_STEP_EVENTS", "1")
    K = args.steps
    marks = set() if mode == "0" else (set(range(K + 1)) if mode == "all" else
                                        set(range(min(6, K + 1))) | set(range(max(0, K - 5), K + 1)))
    evs = {i: torch.cuda.Event(enable_timing=True) for i in marks}
    t0 = time.perf_counter()
    if 0 in evs:
        evs[0].record()
    for i in range(args.steps):
        step()
        if i + 1 in evs:
            evs[i + 1].record()
    # the exchange is queued right behind the last step (no host sync in between, as an optimise loop
    # would run it); its time is the stream time from the last step's end to the exchange's end
    # (pack + all_gather + the header read), from events on the step's stream
    eg0, eg1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    eg0.record()
    buf, records, bufs = exchange()
    n_records = int(records.shape[0])
    eg1.record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    # informational: the same exchange repeated outside the timed region (median host wall time)
    reps = []
    for _ in range(int(os.environ.get("CDX_BENCH_EXCHANGE_REPEAT", "10"))):
        torch.cuda.synchronize()
        tr = time.perf_counter()
        _b, _r, _bs = exchange()
        int(_r.shape[0])
        torch.cuda.synchronize()
        reps.append(time.perf_counter() - tr)
    ms = (ctypes.c_double * N.PROF_STAGES)()
    cnt = (ctypes.c_int64 * N.PROF_STAGES)()
    N.check(lib.cdx_profile_read(ms, cnt), "cdx_profile_read")
    # stage split (informational): every stage timed over a short extra pass, outside the timed region
    ms_all = (ctypes.c_double * N.PROF_STAGES)()
    cnt_all = (ctypes.c_int64 * N.PROF_STAGES)()
    N.check(lib.cdx_profile_enable((1 << N.PROF_STAGES) - 1), "cdx_profile_enable")
    for _ in range(min(10, args.steps)):
        step()
    torch.cuda.synchronize()
    N.check(lib.cdx_profile_read(ms_all, cnt_all), "cdx_profile_read")
    lib.cdx_profile_enable(0)
    live = [bool(cnt[i]) for i in range(N.PROF_STAGES)]  # stages timed inside the timed steps
    for i in range(N.PROF_STAGES):
        if not cnt[i]:
            ms[i], cnt[i] = ms_all[i], cnt_all[i]
    elapsed, gather_s = t1 - t0, eg0.elapsed_time(eg1) * 1e-3
    if world > 1:
        t = torch.tensor([elapsed, gather_s], dtype=torch.float64, device=dev if args.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, gather_s = float(t[0]), float(t[1])
    nan_candidates = int((~torch.isfinite(opt.total_loss)).sum())

    step_ms = [evs[i].elapsed_time(evs[i + 1]) for i in range(K) if i in evs and i + 1 in evs]
    ms_per_step = 1e3 * elapsed / args.steps
    value = E * world / (elapsed / args.steps)
    stage_names = ["queries", "gpis_mean", "gpis_std_var", "cost_bwd", "gpis_std_grad", "gpis_screen"]
    stage_ms = {n: (ms[i] / cnt[i] if cnt[i] else None) for i, n in enumerate(stage_names)}
    lq = opt.problem(gpis, 1).n_query_levels
    m_std, m_grad = lq * E * 4, lq * E
    scr = opt.screen_stats(gpis, E)  # rows of the exact fp64 pass (screened closure), None: all m_std
    m_exact = scr["exact_rows"] if scr else m_std
    n_ind = args.n_inducing
    # algorithmic flops per launch (unpadded N): V = K*·L⁻ᵀ is triangular, N(N+1)/2 MACs per
    # query; W = V·L⁻¹ (= (E11⁻¹k)ᵀ) at the variance cost's argmax fingertip only, also triangular;
    # the screen runs the triangular product for every all-tip row as 3 fp16 slice products
    tri = float(n_ind) * (n_ind + 1)
    flops, flops_g, flops_s = m_exact * tri, m_grad * tri, 3 * m_std * tri
    # algorithmic HBM bytes per launch: the triangle of L⁻ᵀ / L⁻¹ read once (f64), the V rows the
    # refine pass writes / the ∇std pass reads (N_pad f64 each), the screen's fp16 slice pair of the
    # scaled L⁻ᵀ triangle plus its stripe partials (8 f64 per row); queries and outputs are < 1 %
    n_pad = (n_ind + 255) // 256 * 256
    tri_bytes = 8.0 * n_ind * (n_ind + 1) / 2
    alg_refine = tri_bytes + 8.0 * m_exact * n_pad
    alg_grad = tri_bytes + 8.0 * m_grad * n_pad
    alg_screen = 4.0 * n_ind * (n_ind + 1) / 2 + 8.0 * m_std * (n_pad // 256)
    std_ms, grad_ms, scr_ms = stage_ms["gpis_std_var"], stage_ms["gpis_std_grad"], stage_ms["gpis_screen"]
    achieved = flops / (std_ms * 1e-3) / 1e12 if std_ms else None
    achieved_g = flops_g / (grad_ms * 1e-3) / 1e12 if grad_ms else None
    achieved_s = flops_s / (scr_ms * 1e-3) / 1e12 if scr_ms else None

    if rank == 0:
        out = {
            "metric": "candidate-grasp cost+grad evals/sec (GPIS+FK+SDF), 1/2/4/8 GPU",
            "value": value, "unit": "evals/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f64", "data": "synthetic",
            "config": {"workload": (f"config {'2' if world == 1 else '3'}: prob-mode closure fwd+bwd, "
                                    f"{E} candidates/GPU, {args.hand} FK (f32), 3 pregrasp levels; one object per GPU "
                                    f"({', '.join(CONFIG3[:world])}), each an N={n_ind} GPIS (in-repo fit recipe; "
                                    f"rank 0 = config 2's banana); ends with one all_gather of surviving grasps"),
                       "candidates_per_gpu": E, "n_inducing": n_ind, "hand": args.hand,
                       "parallelism": f"one object per GPU over {world} GPU(s), survivors all-gathered"},
            "exchange": {"collective": "all_gather" if world > 1 else None,
                         "backend": (args.backend if world > 1 else None), "ms": gather_s * 1e3,
                         "bytes_per_rank": int(buf.numel() * 8), "records_gathered": n_records,
                         "overflow": D.overflow(bufs),
                         "ms_repeat_median": (1e3 * sorted(reps)[len(reps) // 2]) if reps else None,
                         "note": "pack (cdx_pack_survivors: per-tile counts + rows, two launches, device "
                                 "compaction, header counts on device) + the shape check (one all_reduce, N > 1) "
                                 "+ all_gather + unpack (the one host read of "
                                 "the headers), inside the timed region, queued behind the last step (ms: HIP events on the step stream "
                                 "from the last step's end to the exchange's end); ms_repeat_median: the same "
                                 "exchange repeated after the timed region, host wall time with a sync before each "
                                 "(informational)"},
            "step_ms": ({"min": min(step_ms), "median": statistics.median(step_ms), "max": max(step_ms),
                         "first5_mean": statistics.fmean(step_ms[:5]), "last5_mean": statistics.fmean(step_ms[-5:]),
                         "steps_marked": len(step_ms), **({"all": step_ms} if mode == "all" else {}),
                         "note": "rank 0's stream time of the first and last 5 timed steps (HIP events between "
                                 "them): the clock ramp shows as first5_mean > last5_mean"} if step_ms else None),
            "native": N.build_info(),
            "stage_ms": stage_ms,
            "stage_ms_note": "gpis_std_var (the refine kernel, the headline roofline): HIP events over "
                              "the timed steps; the other stages from a 10-step all-stage pass after the timed "
                              "region; the selection / merge / finalize kernels between them are in no stage; "
                              "gpis_mean runs on a side stream concurrently with the selection, exact-pass and "
                              "merge kernels (screened closure), so its stage time is wall time shared with them",
            "roofline_refine": {"bound": "mfma",
                                "kernel": ("gpis_std_kernel<VARL> (v_mfma_f64_16x16x4_f64, K*·L⁻ᵀ, screened rows)" if scr
                                           else "gpis_std_kernel<VAR> (v_mfma_f64_16x16x4_f64, K*·L⁻ᵀ)"),
                                "achieved": achieved, "peak": FP64_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                                "frac": (achieved / FP64_MFMA_PEAK_TFLOPS) if achieved else None,
                                **traffic_block(E, n_ind, "gpis_refine_bytes_per_launch" if scr
                                                else "gpis_var_bytes_per_launch", alg_refine),
                                "flops_per_launch": flops, "ms": std_ms,
                                "note": f"{m_exact} of {m_std} all-tip rows x N(N+1) in the exact fp64 whitened "
                                        f"form (triangular; all-tip queries deduplicated over the 3 identical "
                                        f"pregrasp levels, the reference does 3x)"},
            "roofline_grad": {"bound": "mfma", "kernel": "gpis_std_kernel<GRADV> (V·L⁻¹ = (E11⁻¹k)ᵀ, ∇std)",
                              "achieved": achieved_g, "peak": FP64_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                              "frac": (achieved_g / FP64_MFMA_PEAK_TFLOPS) if achieved_g else None,
                              **traffic_block(E, n_ind, "gpis_grad_bytes_per_launch", alg_grad),
                              "flops_per_launch": flops_g,
                              "note": f"{m_grad} queries (the variance cost's argmax fingertip) x N(N+1), "
                                      f"from the whitened vectors the std pass keeps"},
            "nan_candidates": nan_candidates,  # reference semantics: unclamped log in :708-709
        }
        if scr:
            out["roofline_screen"] = {
                "bound": "mfma", "kernel": "gpis_screen_kernel (v_mfma_f32_32x32x16_f16, 2-slice fp16 split of "
                                           "(K*−k0)·L⁻ᵀ, 3 slice products)",
                "achieved": achieved_s, "peak": F16_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": (achieved_s / F16_MFMA_PEAK_TFLOPS) if achieved_s else None,
                **traffic_block(E, n_ind, "gpis_screen_bytes_per_launch", alg_screen),
                "flops_per_launch": flops_s, "ms": scr_ms,
                "note": f"{m_std} all-tip rows x 3 x N(N+1) fp16 MFMA flops (the split-precision estimate that "
                        f"selects the rows of the exact pass)"}
            rep = opt.screen_report(gpis, E)
            out["screen"] = {k: rep[k] for k in ("exact_rows", "screened_rows", "audited_rows", "bound_misses",
                                                  "audit_misses", "audit_flips", "faults", "max_ratio",
                                                  "max_ratio_audit", "cum_closures", "cum_audited_rows",
                                                  "cum_bound_misses", "cum_audit_misses", "cum_audit_flips",
                                                  "cum_faults", "cum_max_ratio", "cum_max_ratio_audit", "repaired",
                                                  "discarded_rows", "min_gap", "audit_cut", "cum_repairs",
                                                  "cum_discarded_rows", "cum_min_gap")}
            out["screen"] = {k: (None if isinstance(v, float) and not np.isfinite(v) else v)  # strict JSON: no inf
                             for k, v in out["screen"].items()}
            out["screen"]["delta_over_k0"] = gpis.native_state().desc.screen_delta / float(gpis.R) ** 3
            out["screen"]["note"] = ("every closure re-checks its kept rows and the discarded rows nearest the keep "
                                     "threshold (smallest z = margins below the group's floor) with the exact fp64 "
                                     "pass and repairs itself (every row exact) if a check fails; max_ratio = max "
                                     "|estimate − exact| / margin; min_gap = smallest z left unaudited; cum_* over all "
                                     "closures of this run")
        # the dominant kernel (longest per launch) is the headline roofline
        # the headline roofline: the longest-per-launch kernel among those timed live in the timed steps
        stage_of = {"roofline_refine": 2, "roofline_grad": 4, "roofline_screen": 5}
        for k, i in stage_of.items():
            if k in out:
                out[k]["timed"] = "live, timed steps" if live[i] else "post pass (10 steps after the timed region)"
        cands = [k for k in stage_of if k in out and out[k]["achieved"] and live[stage_of[k]]]
        dom = max(cands, key=lambda k: out[k]["flops_per_launch"] / out[k]["achieved"]) if cands else "roofline_refine"
        out["roofline"] = dict(out[dom], which=dom)
        if world == 1 and not args.no_config4:
            out["config4_kin"] = config4_kin(args, dev)
            out["config4_closure"] = config4_closure(args, dev, gpis)
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args, ref_q, cfg)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
