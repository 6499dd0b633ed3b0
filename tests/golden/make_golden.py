"""Generates the committed golden fixtures by running the REFERENCE itself on CPU.

Container-only (needs ``/root/reference``): ``python tests/golden/make_golden.py``.
The outputs (``tests/golden/*.npz``) are data — seeded inputs and the reference's
outputs on them — and are what pins ``oracle/``.  Nothing from the
reference is copied; it is imported and executed via ``_refload.py``.

Fixtures:
  gpis_<state>.npz    GPIS.pred mean/std, compute_normal, and d(cm·mean + cs·std)/dX at
                      seeded queries (gpis.py:43-87), for the 7 stored states and the
                      N = 2000 synthetic banana state (SURVEY §8d recipe; its X1/y/noise
                      are saved so the state can be refit without the reference).
  fk_<robot>_<mode>.npz  compute_forward_kinematics pos/quat and d(cot·pos)/dq
                      (robot_model.py:224-264) for Allegro, Leap, iiwa7_allegro; recursive=False
                      only (the prob path, optimize_pregrasp.py:665).  recursive=True composes
                      with each body's stale ``self.pose`` from the previous call
                      (rigid_body.py:111-118) and is used only by out-of-scope optimizers.
  closure_<case>.npz  ProbabilisticGraspOptimizer.closure (optimize_pregrasp.py:741-769):
                      inputs, the captured Kabsch noise (``rand_like`` at :61), total_loss,
                      total_margin, pregrasp tips and the 5 parameter gradients.
  optimize_<case>.npz ProbabilisticGraspOptimizer.optimize (:771-839) for 30 iterations
                      with a replayed noise sequence.
  collision_<hand>.npz compute_collision_loss (:671-701) cost and d(Σ cost)/d(q, palm pose).
  force_eq_<case>.npz force_eq_reward (:73-118) outputs and input gradients, noise captured.
  mode_<mode>.npz     GPIS / KinGPIS / SDF / Kin optimisers (:121-511), 12 iterations, E = 6: final
                      outputs and the per-iteration Σ loss (TorchSDF via the C oracle, whose _C
                      module the reference lacks).
  gpis_box.npz        as gpis_<state> for config 3's box object (no stored state: fitted by the
                      reference GPIS.fit on compliancedex_amd.workloads.box_arrays; X1/y/noise saved).
  normals_<state>.npz compute_normal(X, index) (gpis.py:63-87, index branch: normals + Σ weights)
                      for three index sets, and compute_multinormals (:89-111) for 3 and 5 samples,
                      2-D and 3-D query batches.
  closure_iiwa7_*.npz the prob closure on the 23-DOF iiwa7_allegro chain (config 4) plus
                      compute_collision_loss (:671-701) on the same inputs (the reference closure has
                      it commented out at :765; the build's collision=True adds it).
  results_<exp>.npz   the reference's own optimiser outputs data/{contact,target,wrist,compliance,
                      joint_angle}_<exp>.npy (writer :1016-1020), copied as data for the FK/format check.
"""
from __future__ import annotations

import contextlib
import io
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import _refload  # noqa: E402

OUT = HERE
STATES = ["banana", "coffeebottle", "hammer", "lego", "mug", "mug2", "dummy"]


def obj_vertices(path):
    vs = []
    with open(path) as f:
        for line in f:
            if line.startswith("v "):
                vs.append([float(x) for x in line.split()[1:4]])
    return np.asarray(vs)


class NoiseTape:
    """Replaces torch.rand_like on the Kabsch path with a recorded / replayed stream."""

    def __init__(self, torch, seed=0, replay=None):
        self.torch = torch
        self.gen = torch.Generator().manual_seed(seed)
        self.replay = list(replay) if replay is not None else None
        self.record = []
        self._orig = torch.rand_like

    def __enter__(self):
        torch = self.torch

        def rand_like(t, *a, **k):
            if self.replay is not None:
                out = self.replay.pop(0).to(t.dtype)
            else:
                out = torch.rand(t.shape, dtype=t.dtype, generator=self.gen)
            self.record.append(out.clone())
            return out

        torch.rand_like = rand_like
        return self

    def __exit__(self, *exc):
        self.torch.rand_like = self._orig


def load_state(ns, name):
    g = ns.gpis.GPIS(0.08, 1.0)
    cwd = os.getcwd()
    os.chdir(ns.ref)
    try:
        g.load_state_data(f"{name}_state")
    finally:
        os.chdir(cwd)
    return g


def synthetic_banana(ns, n_total=2000):
    """SURVEY §8d recipe, following optimize_pregrasp.py:904-922."""
    torch = ns.torch
    pcd = np.load(os.path.join(ns.ref, "partial_pcd/banana.npy"))
    center = 0.5 * (pcd.min(0) + pcd.max(0))
    n_ext, n_int = 14, 50
    n_surf = n_total - n_ext - n_int
    rng = np.random.default_rng(0)
    surf = pcd[rng.permutation(len(pcd))[:n_surf]]
    bound = 0.15
    ext = np.array([[-1, -1, -1], [1, -1, -1], [-1, 1, -1], [1, 1, -1],
                    [-1, -1, 1], [1, -1, 1], [-1, 1, 1], [1, 1, 1],
                    [-1, 0, 0], [0, -1, 0], [1, 0, 0], [0, 1, 0],
                    [0, 0, 1], [0, 0, -1]], dtype=np.float64) * bound + center
    gen = torch.Generator().manual_seed(0)
    w = torch.rand(n_int, n_surf, generator=gen).double()
    internal = (torch.softmax(w * 30, dim=1) @ torch.from_numpy(surf)).numpy()
    X1 = np.vstack([ext, surf, internal])
    y = np.concatenate([np.full(n_ext, bound), np.zeros(n_surf), np.full(n_int, -bound)])[:, None]
    noise = np.concatenate([np.full(n_ext, 0.2), np.full(n_surf, 0.005), np.full(n_int, 0.1)])
    g = ns.gpis.GPIS(0.08, 1.0)
    g.fit(torch.from_numpy(X1), torch.from_numpy(y), noise=torch.from_numpy(noise))
    g.bias = torch.tensor(1.0, dtype=torch.float64)
    return g, dict(syn_X1=X1, syn_y=y, syn_noise=noise)


def gen_gpis(ns):
    torch = ns.torch
    rng = np.random.default_rng(1)
    cases = [(s, load_state(ns, s), {}) for s in STATES]
    g, extra = synthetic_banana(ns)
    cases.append(("synthetic2000", g, extra))
    for name, g, extra in cases:
        X1 = g.X1.numpy()
        lo, hi = X1.min(0) - 0.03, X1.max(0) + 0.03
        M = 96
        Xq = lo + (hi - lo) * rng.random((M, 3))
        # include a few points ON training points (exact-surface case) and near them
        Xq[:4] = X1[rng.integers(0, len(X1), 4)] + 1e-4 * rng.standard_normal((4, 3))
        X = torch.from_numpy(Xq).requires_grad_(True)
        mean, std = g.pred(X)
        cm = rng.standard_normal(M)
        cs = rng.standard_normal(M)
        (mean * torch.from_numpy(cm)).sum().add((std * torch.from_numpy(cs)).sum()).backward()
        normal = g.compute_normal(torch.from_numpy(Xq))
        # batched 3-D input path (gpis.py:48-50): [M/4, 4, 3] -> [M/4, 4]
        mean3, std3 = g.pred(torch.from_numpy(Xq).view(-1, 4, 3))
        np.savez_compressed(
            os.path.join(OUT, f"gpis_{name}.npz"),
            X=Xq, mean=mean.detach().numpy(), std=std.detach().numpy(), cm=cm, cs=cs,
            grad_X=X.grad.numpy(), normal=normal.numpy(),
            mean3=mean3.detach().numpy(), std3=std3.detach().numpy(),
            R=float(g.R), bias=float(g.bias), **extra)
        print("gpis", name, len(X1))


def gen_fk(ns):
    torch = ns.torch
    rng = np.random.default_rng(2)
    ee_offsets = ns.opt.EE_OFFSETS
    specs = [
        ("allegro", ns.robot_configs["allegro"]["ee_link_name"], ns.robot_configs["allegro"]["ee_link_offset"].tolist(),
         ns.robot_configs["allegro"]["ref_q"], "cfg"),
        ("allegro", ns.robot_configs["allegro"]["ee_link_name"], ee_offsets, ns.robot_configs["allegro"]["ref_q"], "eeoff"),
        ("leap", ns.robot_configs["leap"]["ee_link_name"], ns.robot_configs["leap"]["ee_link_offset"].tolist(),
         ns.robot_configs["leap"]["ref_q"], "cfg"),
        ("iiwa7_allegro", ["link_3.0_tip", "link_7.0_tip", "link_11.0_tip", "link_15.0_tip"], ee_offsets, None, "eeoff"),
    ]
    for robot, links, offsets, ref_q, tag in specs:
        model = ns.rm.DifferentiableRobotModel(os.path.join(ns.ref, _refload.URDFS[robot]))
        B = 32
        dof = model._n_dofs
        base = np.zeros(dof) if ref_q is None else np.asarray(ref_q)
        scale = 0.3 if ref_q is None else 0.1
        q = (base + scale * rng.standard_normal((B, dof))).astype(np.float32)
        for recursive in (False,):
            qt = torch.from_numpy(q).requires_grad_(True)
            with contextlib.redirect_stdout(io.StringIO()):
                pos, quat = model.compute_forward_kinematics(qt, links, recursive=recursive, offsets=offsets)
            cot = rng.standard_normal(pos.shape).astype(np.float32)
            (pos * torch.from_numpy(cot)).sum().backward()
            mode = "rec" if recursive else "nonrec"
            np.savez_compressed(
                os.path.join(OUT, f"fk_{robot}_{tag}_{mode}.npz"),
                q=q, pos=pos.detach().numpy(), quat=quat.detach().numpy(), cot=cot,
                grad_q=qt.grad.numpy(), links=np.array(links), offsets=np.asarray(offsets, dtype=np.float64))
            print("fk", robot, tag, mode)


def problem_inputs(ns, hand, E, seed, perturb_target):
    """Mirrors optimize_pregrasp.py __main__ (:872-999) with --use_config, headless.

    The object centre is the banana mesh's vertex AABB centre (the reference uses the
    AABB of a random Poisson sample of the same mesh, :885-888)."""
    torch = ns.torch
    cfg = {"wrist_x": 0.0, "wrist_y": 0.015, "wrist_z": 0.11, "floor_offset": 0.02}
    verts = obj_vertices(os.path.join(ns.ref, "assets/banana/banana.obj"))
    center = 0.5 * (verts.min(0) + verts.max(0))
    W = np.array(ns.opt.WRIST_OFFSET, dtype=np.float64).copy()
    W[:, 0] += center[0]
    W[:, 1] += center[1]
    W[:, 2] += 2 * center[2]
    W[:, 0] += cfg["wrist_x"]
    W[:, 1] += cfg["wrist_y"]
    W[:, 2] += cfg["wrist_z"] - cfg["floor_offset"]
    rng = np.random.default_rng(seed)
    idx = np.arange(E) % len(W)
    palm = W[idx]
    ref_q = np.asarray(ns.robot_configs[hand]["ref_q"], dtype=np.float64)
    q = np.tile(ref_q, (E, 1))
    target = np.tile(center, (E, 4, 1)).astype(np.float64)
    if E > len(W):
        q = q + 0.1 * rng.standard_normal(q.shape)
        palm = palm + np.concatenate([0.005 * rng.standard_normal((E, 3)), 0.05 * rng.standard_normal((E, 3))], 1)
    if perturb_target:
        target = target + 0.01 * rng.standard_normal(target.shape)
    comp = np.tile(np.array([10.0, 10.0, 10.0, 20.0]), (E, 1))
    return dict(q=q, comp=comp, target=target, palm=palm, center=center, W=W)


def make_optimizer(ns, hand, palm, num_iters):
    rc = ns.robot_configs[hand]
    with contextlib.redirect_stdout(io.StringIO()):
        o = ns.opt.ProbabilisticGraspOptimizer(
            os.path.join(ns.ref, _refload.URDFS[hand]),
            ee_link_names=rc["ee_link_name"], ee_link_offsets=rc["ee_link_offset"].tolist(),
            anchor_link_names=rc["collision_links"], anchor_link_offsets=rc["collision_offsets"].tolist(),
            collision_pairs=rc["collision_pairs"],
            tip_bounding_box=[ns.opt.FINGERTIP_LB, ns.opt.FINGERTIP_UB],
            ref_q=rc["ref_q"].tolist(), optimize_target=True, optimize_palm=True,
            num_iters=num_iters, palm_offset=palm, mass=0.1, com=[0.0, 0.0, 0.0],
            gravity=True, uncertainty=20.0)
    return o


def gen_closure(ns, name, hand, state, E, seed, perturb_target, gpis_obj=None):
    torch = ns.torch
    inp = problem_inputs(ns, hand, E, seed, perturb_target)
    g = gpis_obj if gpis_obj is not None else load_state(ns, state)
    o = make_optimizer(ns, hand, inp["palm"], 1)
    q = torch.from_numpy(inp["q"]).clone().requires_grad_(True)
    comp = torch.from_numpy(inp["comp"]).clone().requires_grad_(True)
    target = torch.from_numpy(inp["target"]).clone().requires_grad_(True)
    palm_pos = torch.from_numpy(inp["palm"][:, :3]).clone().requires_grad_(True)
    palm_ori = torch.from_numpy(inp["palm"][:, 3:]).clone().requires_grad_(True)
    o.optim = torch.optim.Adam([q, comp, target, palm_pos, palm_ori])
    with NoiseTape(torch, seed=seed) as tape, contextlib.redirect_stdout(io.StringIO()):
        loss = o.closure(q, comp, target, palm_pos, palm_ori, 1, g, E)
    noise = torch.stack(tape.record).numpy()
    np.savez_compressed(
        os.path.join(OUT, f"closure_{name}.npz"),
        hand=hand, state=state, q=inp["q"], comp=inp["comp"], target=inp["target"], palm=inp["palm"],
        center=inp["center"], noise=noise, loss=float(loss), total_loss=o.total_loss.detach().numpy(),
        total_margin=o.total_margin.detach().numpy(), pregrasp_tip=o.pregrasp_tip_pose.detach().numpy(),
        grad_q=q.grad.numpy(), grad_comp=comp.grad.numpy(), grad_target=target.grad.numpy(),
        grad_palm_pos=palm_pos.grad.numpy(), grad_palm_ori=palm_ori.grad.numpy())
    print("closure", name, float(loss))


def gen_optimize(ns, name, hand, state, E, seed, iters):
    torch = ns.torch
    inp = problem_inputs(ns, hand, E, seed, False)
    g = load_state(ns, state)
    o = make_optimizer(ns, hand, inp["palm"], iters)
    gen = torch.Generator().manual_seed(seed)
    tape = [torch.rand((3 * E, 3, 3), dtype=torch.float64, generator=gen) for _ in range(iters)]
    trace = []
    closure = o.closure

    def traced(*a, **k):  # per-iteration total_loss: the input of the best-iterate update_flag (:821-829)
        r = closure(*a, **k)
        trace.append(o.total_loss.detach().clone())
        return r
    o.closure = traced
    with NoiseTape(torch, replay=tape), contextlib.redirect_stdout(io.StringIO()):
        out = o.optimize(torch.from_numpy(inp["q"]), torch.from_numpy(inp["target"]),
                         torch.from_numpy(inp["comp"]), 1, g)
    opt_q, opt_comp, opt_target, opt_palm, opt_margin = [t.detach().numpy() for t in out]
    np.savez_compressed(
        os.path.join(OUT, f"optimize_{name}.npz"),
        hand=hand, state=state, iters=iters, q=inp["q"], comp=inp["comp"], target=inp["target"],
        palm=inp["palm"], noise=torch.stack(tape).numpy(), opt_q=opt_q, opt_comp=opt_comp,
        opt_target=opt_target, opt_palm=opt_palm, opt_margin=opt_margin, loss_trace=torch.stack(trace).numpy())
    print("optimize", name)


def gen_force_eq(ns, name, B, seed, gravity, mu, mass=0.1, com=(0.0, 0.0, 0.0)):
    """force_eq_reward (:73-118) on seeded rows: reward, margin, force_norm and
    d(Σ cr·reward + Σ cf·force_norm)/d(tip, target, compliance); Kabsch noise captured.  Half the
    rows put the tips close to their targets (near-rank-1 H, as at the optimisers' start)."""
    torch = ns.torch
    rng = np.random.default_rng(seed)
    T = 4
    target = 0.05 * rng.standard_normal((B, T, 3))
    tip = target + 0.03 * rng.standard_normal((B, T, 3))
    tip[: B // 2] = target[: B // 2] + 1e-3 * rng.standard_normal((B // 2, T, 3))
    comp = rng.uniform(10.0, 200.0, (B, T))
    normal = rng.standard_normal((B, T, 3))
    normal /= np.linalg.norm(normal, axis=2, keepdims=True)
    cr, cf = rng.standard_normal(B), rng.standard_normal((B, T))
    tt = torch.from_numpy(tip).clone().requires_grad_(True)
    gt = torch.from_numpy(target).clone().requires_grad_(True)
    ct = torch.from_numpy(comp).clone().requires_grad_(True)
    with NoiseTape(torch, seed=seed) as tape:
        reward, margin, fn = ns.opt.force_eq_reward(tt, gt, ct, mu, torch.from_numpy(normal), mass=mass,
                                                    gravity=10.0 if gravity else None, COM=list(com))
    ((reward * torch.from_numpy(cr)).sum() + (fn * torch.from_numpy(cf)).sum()).backward()
    np.savez_compressed(os.path.join(OUT, f"force_eq_{name}.npz"), tip=tip, target=target, comp=comp, normal=normal,
                        noise=torch.stack(tape.record).numpy().reshape(B, 9), gravity=gravity, mu=mu, mass=mass,
                        com=np.asarray(com), cr=cr, cf=cf, reward=reward.detach().numpy(),
                        margin=margin.detach().numpy(), force_norm=fn.detach().numpy(), grad_tip=tt.grad.numpy(),
                        grad_target=gt.grad.numpy(), grad_comp=ct.grad.numpy())
    print("force_eq", name, float(reward.sum()))


class _OracleSDF:
    """CPU compute_sdf for the reference's SDF / Kin optimisers (its CUDA _C module is absent):
    the C oracle (oracle/sdf_oracle.c, the restatement pinned in tests/test_sdf_cpu.py) forward,
    backward 2·g·(p − c) as unbatched_triangle_distance_cuda.cu:263-269."""

    def __init__(self, torch):
        sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
        from tests import _sdf_oracle
        self.o = _sdf_oracle
        o = _sdf_oracle

        class Fn(torch.autograd.Function):
            @staticmethod
            def forward(ctx, points, faces):
                assert points.dtype == torch.float32 and faces.dtype == torch.float32
                d, sg, n, c, _ = o.forward(points.detach().numpy(), faces.detach().numpy())
                c = torch.from_numpy(c)
                ctx.save_for_backward(points.detach(), c)
                sg, n = torch.from_numpy(sg), torch.from_numpy(n)
                ctx.mark_non_differentiable(sg, n, c)
                return torch.from_numpy(d), sg, n, c

            @staticmethod
            def backward(ctx, g, *_):
                p, c = ctx.saved_tensors
                return torch.from_numpy(o.backward(g.contiguous().numpy(), p.numpy(), c.numpy())), None

        self.fn = Fn

    def __call__(self, points, faces):
        return self.fn.apply(points, faces)


def _loss_trace(text):
    out = []
    for line in text.splitlines():
        if line.startswith("Loss:"):
            out.append(float(line.split()[1].rstrip(",")))
    return np.asarray(out)


def gen_modes(ns, iters=12, E=6, seed=50):
    """The four other optimisers (:121-511) for ``iters`` iterations on the banana, noise replayed;
    final outputs + the per-iteration Σ loss parsed from their verbose prints."""
    torch = ns.torch
    from compliancedex_amd.optimizers import TriangleMesh
    ns.opt.compute_sdf = _OracleSDF(torch)
    rng = np.random.default_rng(seed)
    verts = obj_vertices(os.path.join(ns.ref, "assets/banana/banana.obj"))
    center = 0.5 * (verts.min(0) + verts.max(0))
    init_tip = np.array([[0.05, 0.05, 0.02], [0.06, -0.0, -0.01], [0.03, -0.04, 0.0], [-0.07, -0.01, 0.02]])
    tips = center + init_tip + 0.005 * rng.standard_normal((E, 4, 3))
    target = np.tile(center, (E, 4, 1)) + 0.003 * rng.standard_normal((E, 4, 3))
    comp = np.tile([10.0, 10.0, 10.0, 20.0], (E, 1))
    rc = ns.robot_configs["allegro"]
    q = np.asarray(rc["ref_q"], dtype=np.float64) + 0.05 * rng.standard_normal((E, 16))
    palm3 = np.array([-0.06 + center[0], 0.015 + center[1], 0.05 + 2 * center[2] + 0.09])
    bbox = [ns.opt.FINGERTIP_LB, ns.opt.FINGERTIP_UB]
    links, offs = rc["ee_link_name"], rc["ee_link_offset"].tolist()
    urdf = os.path.join(ns.ref, _refload.URDFS["allegro"])

    def mesh():
        vs, fs = [], []
        for line in open(os.path.join(ns.ref, "assets/banana/banana.obj")):
            if line.startswith("f "):
                fs.append([int(t.split("/")[0]) - 1 for t in line.split()[1:4]])
        return TriangleMesh(verts, fs)

    def run(name, f32, make, call):
        nonlocal E
        dt = torch.float32 if f32 else torch.float64
        gen = torch.Generator().manual_seed(seed)
        tape = [torch.rand((E, 3, 3), dtype=dt, generator=gen).double() for _ in range(iters)]
        with NoiseTape(torch, replay=tape) as nt, contextlib.redirect_stdout(io.StringIO()) as buf:
            o = make()
            out = call(o, dt)
        trace = _loss_trace(buf.getvalue())
        assert len(trace) == iters, (name, len(trace))
        res = [t.detach().double().numpy() for t in out[:3]]
        np.savez_compressed(os.path.join(OUT, f"mode_{name}.npz"), mode=name, iters=iters, tips=tips, target=target,
                            comp=comp, q=q, palm3=palm3, center=center, noise=torch.stack(nt.record).numpy(),
                            f32=f32, out0=res[0], out1=res[1], out2=res[2], flag=bool(out[3]), loss_trace=trace)
        print("mode", name, trace[0], trace[-1], bool(out[3]))

    g = load_state(ns, "banana")
    run("gpis", False, lambda: ns.opt.GPISGraspOptimizer(bbox, num_iters=iters, optimize_target=True),
        lambda o, dt: o.optimize(torch.from_numpy(tips), torch.from_numpy(target), torch.from_numpy(comp), 1, g))
    run("kingpis", False,
        lambda: ns.opt.KinGPISGraspOptimizer(urdf, links, offs, palm_offset=palm3.tolist(), num_iters=iters,
                                             optimize_target=True, ref_q=rc["ref_q"].tolist(), tip_bounding_box=bbox),
        lambda o, dt: o.optimize(torch.from_numpy(q), torch.from_numpy(target), torch.from_numpy(comp), 1, g))
    # SDF / Kin modes: the reference broadcasts tar_sign [E·T] against a [E, T] view (:297, :211), which
    # only runs for E = 1 — one candidate each
    E = 1
    tips, target, comp, q = tips[:1], target[:1], comp[:1], q[:1]
    run("sdf", True, lambda: ns.opt.SDFGraspOptimizer(bbox, num_iters=iters, optimize_target=True),
        lambda o, dt: o.optimize(torch.from_numpy(tips).float(), torch.from_numpy(target).float(),
                                 torch.from_numpy(comp).float(), 1, mesh()))
    run("kin", True,
        lambda: ns.opt.KinGraspOptimizer(urdf, links, offs, palm_offset=palm3.tolist(), num_iters=iters,
                                         optimize_target=True, ref_q=rc["ref_q"].tolist()),
        lambda o, dt: o.optimize(torch.from_numpy(q).float(), torch.from_numpy(target).float(),
                                 torch.from_numpy(comp).float(), 1, mesh()))


def gen_collision(ns, name, hand, E, seed):
    """compute_collision_loss (:671-701) with its autograd gradient w.r.t. q and the palm pose.
    Joint angles are perturbed hard and palm heights drawn low so the pairwise (< 0.02), anchor
    floor (z < 0.02) and palm floor terms all fire on some candidates."""
    torch = ns.torch
    inp = problem_inputs(ns, hand, E, seed, True)
    rng = np.random.default_rng(seed + 100)
    q = inp["q"] + 0.6 * rng.standard_normal(inp["q"].shape)
    palm = inp["palm"].copy()
    palm[:, 2] = rng.uniform(0.004, 0.09, E)
    o = make_optimizer(ns, hand, palm, 1)
    qt = torch.from_numpy(q).clone().requires_grad_(True)
    pt = torch.from_numpy(palm).clone().requires_grad_(True)
    with contextlib.redirect_stdout(io.StringIO()):
        cost = o.compute_collision_loss(qt, pt)
    cost.sum().backward()
    np.savez_compressed(os.path.join(OUT, f"collision_{name}.npz"), hand=hand, q=q, palm=palm,
                        cost=cost.detach().numpy(), grad_q=qt.grad.numpy(), grad_palm=pt.grad.numpy())
    print("collision", name, int((cost.detach() != 0).sum()), "of", E, "non-zero")


def gen_gpis_box(ns):
    """Config 3's box GPIS: the reference GPIS.fit on the build's box recipe, pred/normal at
    seeded queries (same fields as gen_gpis, X1/y/noise saved as syn_*)."""
    torch = ns.torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    from compliancedex_amd.workloads import box_arrays
    X1, y, noise = box_arrays()
    g = ns.gpis.GPIS(0.08, 1.0)
    g.fit(torch.from_numpy(X1), torch.from_numpy(y), noise=torch.from_numpy(noise))
    g.bias = torch.tensor(1.0, dtype=torch.float64)
    rng = np.random.default_rng(5)
    M = 96
    lo, hi = X1.min(0) - 0.03, X1.max(0) + 0.03
    Xq = lo + (hi - lo) * rng.random((M, 3))
    # near the cube faces: where the variance cost and the closure's queries live
    Xq[:48] = X1[14 + rng.integers(0, 400, 48)] + 2e-3 * rng.standard_normal((48, 3))
    X = torch.from_numpy(Xq).requires_grad_(True)
    mean, std = g.pred(X)
    cm, cs = rng.standard_normal(M), rng.standard_normal(M)
    (mean * torch.from_numpy(cm)).sum().add((std * torch.from_numpy(cs)).sum()).backward()
    normal = g.compute_normal(torch.from_numpy(Xq))
    mean3, std3 = g.pred(torch.from_numpy(Xq).view(-1, 4, 3))
    np.savez_compressed(os.path.join(OUT, "gpis_box.npz"), X=Xq, mean=mean.detach().numpy(), std=std.detach().numpy(),
                        cm=cm, cs=cs, grad_X=X.grad.numpy(), normal=normal.numpy(), mean3=mean3.detach().numpy(),
                        std3=std3.detach().numpy(), R=float(g.R), bias=float(g.bias), syn_X1=X1, syn_y=y,
                        syn_noise=noise)
    print("gpis box", len(X1))


def gen_normals(ns):
    """compute_normal(X, index) and compute_multinormals on stored states (fresh GPIS object per
    multinormals call: the reference caches ``fraction``/``indices`` from the first call)."""
    torch = ns.torch
    for name, seed in (("banana", 60), ("mug", 61)):
        rng = np.random.default_rng(seed)
        g = load_state(ns, name)
        X1 = g.X1.numpy()
        n = len(X1)
        Xq = X1[rng.integers(0, n, 48)] + 5e-3 * rng.standard_normal((48, 3))
        idx_sets = [list(range(int(0.8 * n))), sorted(rng.choice(n, n // 2, replace=False).tolist()),
                    list(range(n // 3, n))]
        out = dict(X=Xq)
        for i, idx in enumerate(idx_sets):
            nrm, w = g.compute_normal(torch.from_numpy(Xq), idx)
            out[f"index{i}"] = np.asarray(idx)
            out[f"normal_index{i}"] = nrm.numpy()
            out[f"weight_index{i}"] = float(w)
        for S in (3, 5):
            for dim in (2, 3):
                gs = load_state(ns, name)
                X = torch.from_numpy(Xq) if dim == 2 else torch.from_numpy(Xq).view(-1, 4, 3)
                nrms, ws = gs.compute_multinormals(X, S)
                out[f"multi{S}_{dim}d_normals"] = nrms.numpy()
                out[f"multi{S}_{dim}d_weights"] = ws.numpy()
        np.savez_compressed(os.path.join(OUT, f"normals_{name}.npz"), **out)
        print("normals", name, n)


IIWA7_TIPS = ["link_3.0_tip", "link_7.0_tip", "link_11.0_tip", "link_15.0_tip"]
IIWA7_PAIRS = [[0, 1], [0, 2], [0, 3], [1, 2], [1, 3], [2, 3]]


def gen_closure_iiwa7(ns, name, E, seed, gpis_name="banana"):
    """Config 4's chain: the prob closure on iiwa7_allegro (23 DOF; the arm base is the "palm"
    pose, placed so the fingertips at q = 0 surround the banana), fingertips as the collision
    anchors with all six pairs, then compute_collision_loss on the same inputs."""
    torch = ns.torch
    urdf = os.path.join(ns.ref, _refload.URDFS["iiwa7_allegro"])
    offs = [list(o) for o in ns.opt.EE_OFFSETS]
    D = 23
    model = ns.rm.DifferentiableRobotModel(urdf)
    with contextlib.redirect_stdout(io.StringIO()):
        tips0 = model.compute_forward_kinematics(torch.zeros(1, D), IIWA7_TIPS, offsets=offs,
                                                 recursive=False)[0].view(4, 3).double().mean(0).numpy()
    verts = obj_vertices(os.path.join(ns.ref, "assets/banana/banana.obj"))
    center = 0.5 * (verts.min(0) + verts.max(0))
    rng = np.random.default_rng(seed)
    q = 0.3 * rng.standard_normal((E, D))
    q[:, :7] *= 0.1  # the 7 arm joints: small, so the fingertips stay around the object
    palm = np.concatenate([center - tips0 + 0.01 * rng.standard_normal((E, 3)), 0.05 * rng.standard_normal((E, 3))], 1)
    target = np.tile(center, (E, 4, 1)) + 0.01 * rng.standard_normal((E, 4, 3))
    comp = np.tile(np.array([10.0, 10.0, 10.0, 20.0]), (E, 1))
    g = load_state(ns, gpis_name)
    with contextlib.redirect_stdout(io.StringIO()):
        o = ns.opt.ProbabilisticGraspOptimizer(
            urdf, ee_link_names=IIWA7_TIPS, ee_link_offsets=offs, anchor_link_names=IIWA7_TIPS,
            anchor_link_offsets=offs, collision_pairs=IIWA7_PAIRS,
            tip_bounding_box=[ns.opt.FINGERTIP_LB, ns.opt.FINGERTIP_UB], ref_q=[0.0] * D, optimize_target=True,
            optimize_palm=True, num_iters=1, palm_offset=palm, mass=0.1, com=[0.0, 0.0, 0.0], gravity=True,
            uncertainty=20.0)
    qt = torch.from_numpy(q).clone().requires_grad_(True)
    ct = torch.from_numpy(comp).clone().requires_grad_(True)
    tt = torch.from_numpy(target).clone().requires_grad_(True)
    pp = torch.from_numpy(palm[:, :3]).clone().requires_grad_(True)
    po = torch.from_numpy(palm[:, 3:]).clone().requires_grad_(True)
    o.optim = torch.optim.Adam([qt, ct, tt, pp, po])
    with NoiseTape(torch, seed=seed) as tape, contextlib.redirect_stdout(io.StringIO()):
        loss = o.closure(qt, ct, tt, pp, po, 1, g, E)
    noise = torch.stack(tape.record).numpy()
    qc = torch.from_numpy(q).clone().requires_grad_(True)
    pc = torch.from_numpy(palm).clone().requires_grad_(True)
    with contextlib.redirect_stdout(io.StringIO()):
        cost = o.compute_collision_loss(qc, pc)
    cost.sum().backward()
    np.savez_compressed(
        os.path.join(OUT, f"closure_{name}.npz"),
        hand="iiwa7_allegro", state=gpis_name, q=q, comp=comp, target=target, palm=palm, center=center, noise=noise,
        loss=float(loss), total_loss=o.total_loss.detach().numpy(), total_margin=o.total_margin.detach().numpy(),
        pregrasp_tip=o.pregrasp_tip_pose.detach().numpy(), grad_q=qt.grad.numpy(), grad_comp=ct.grad.numpy(),
        grad_target=tt.grad.numpy(), grad_palm_pos=pp.grad.numpy(), grad_palm_ori=po.grad.numpy(),
        links=np.array(IIWA7_TIPS), offsets=np.asarray(offs), pairs=np.asarray(IIWA7_PAIRS),
        coll_cost=cost.detach().numpy(), coll_grad_q=qc.grad.numpy(), coll_grad_palm=pc.grad.numpy())
    print("closure", name, float(loss), "collision non-zero", int((cost.detach() != 0).sum()), "of", E)


def gen_results(ns):
    """The reference's own optimiser outputs (data/*_<exp>.npy), as data for the results check."""
    for exp in ("lego", "realsense"):
        arrs = {k: np.load(os.path.join(ns.ref, "data", f"{k}_{exp}.npy"))
                for k in ("contact", "target", "wrist", "compliance", "joint_angle")}
        np.savez_compressed(os.path.join(OUT, f"results_{exp}.npz"), **arrs)
        print("results", exp, {k: v.shape for k, v in arrs.items()})


def main():
    ns = _refload.load()
    torch = ns.torch
    torch.set_num_threads(8)
    what = sys.argv[1:] or ["gpis", "fk", "closure", "optimize", "collision", "force_eq", "modes", "box", "normals",
                            "iiwa7", "results"]
    if "gpis" in what:
        gen_gpis(ns)
    if "fk" in what:
        gen_fk(ns)
    if "closure" in what:
        gen_closure(ns, "allegro_banana_e6", "allegro", "banana", 6, 10, False)
        gen_closure(ns, "allegro_banana_e64", "allegro", "banana", 64, 11, False)
        gen_closure(ns, "allegro_banana_e64_spread", "allegro", "banana", 64, 12, True)
        gen_closure(ns, "leap_banana_e64", "leap", "banana", 64, 13, False)
        gen_closure(ns, "leap_banana_e64_spread", "leap", "banana", 64, 14, True)
        gen_closure(ns, "allegro_mug_e16_spread", "allegro", "mug", 16, 15, True)
        g, _ = synthetic_banana(ns)
        gen_closure(ns, "allegro_syn2000_e16_spread", "allegro", "synthetic2000", 16, 16, True, gpis_obj=g)
    if "modes" in what:
        gen_modes(ns)
    if "force_eq" in what:
        gen_force_eq(ns, "gravity_mu1", 64, 40, True, 1)
        gen_force_eq(ns, "nogravity_mu05", 64, 41, False, 0.5)
    if "collision" in what:
        gen_collision(ns, "allegro_e64", "allegro", 64, 30)
        gen_collision(ns, "leap_e64", "leap", 64, 31)
    if "optimize" in what:
        gen_optimize(ns, "allegro_banana_e6", "allegro", "banana", 6, 20, 30)
    if "box" in what:
        gen_gpis_box(ns)
    if "normals" in what:
        gen_normals(ns)
    if "iiwa7" in what:
        gen_closure_iiwa7(ns, "iiwa7_banana_e16", 16, 70)
        gen_closure_iiwa7(ns, "iiwa7_mug_e16", 16, 71, gpis_name="mug")
    if "results" in what:
        gen_results(ns)


if __name__ == "__main__":
    main()
