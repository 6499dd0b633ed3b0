"""Drop-ins for the other pregrasp optimisers of optimize_pregrasp.py:

  KinGraspOptimizer      :121-227  joint space, TorchSDF mesh distance, Adam
  SDFGraspOptimizer      :229-320  fingertip space, TorchSDF mesh distance, RMSprop, box clamps
  GPISGraspOptimizer     :322-406  fingertip space, GPIS distance / variance, RMSprop
  KinGPISGraspOptimizer  :408-511  joint space, GPIS distance / log-variance, RMSprop

Each loop runs on the same gfx950 kernels as the prob-mode closure — GPIS mean/normal/std
(cdx_gpis_*), FK (cdx_fk_*), TorchSDF (cdx_sdf_*) and the Kabsch/force-equilibrium reward
(cdx_force_eq_*) — with the per-candidate cost glue as device tensor ops and torch's own
RMSprop / Adam, as in the reference.  Differences in *how*: the best-iterate bookkeeping
(:215-224 etc.) is done with masked device updates instead of ``if update_flag.sum()`` host syncs
(same result: ``opt_margin`` is the margin of the last iteration that improved any candidate);
``kabsch_noise`` (optional, one [E, 3, 3] tensor per iteration) replays the reference's
``rand_like(H)`` draws.  WCKinGPISGraspOptimizer (:513-612) needs cvxpylayers (absent) and is out
of scope.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from . import _native as N
from .force_eq import force_eq_descriptor, force_eq_reward
from .optimizer import EE_OFFSETS, FINGERTIP_LB, FINGERTIP_UB, WRIST_OFFSET
from .robot_model import DifferentiableRobotModel
from .torchsdf import BatchSchedule, PreparedMesh, QueryWorkspace, compute_sdf, query_batch


class TriangleMesh:
    """The part of open3d.geometry.TriangleMesh the SDF optimisers use: ``vertices``,
    ``triangles`` and ``scale(factor, center)`` (in place, like open3d)."""

    def __init__(self, vertices, triangles):
        self.vertices = np.asarray(vertices, dtype=np.float64).copy()
        self.triangles = np.asarray(triangles, dtype=np.int64).copy()

    @classmethod
    def from_npz(cls, path):
        d = np.load(path)
        return cls(d["vertices"], d["triangles"])

    @classmethod
    def from_obj(cls, path):
        vs, fs = [], []
        with open(path) as f:
            for line in f:
                if line.startswith("v "):
                    vs.append([float(x) for x in line.split()[1:4]])
                elif line.startswith("f "):
                    fs.append([int(tok.split("/")[0]) - 1 for tok in line.split()[1:4]])
        return cls(vs, fs)

    def scale(self, factor, center):
        c = np.asarray(center, dtype=np.float64)
        self.vertices = (self.vertices - c) * factor + c
        return self


def _face_vertices(mesh, device):
    tri = np.asarray(mesh.triangles)
    v = np.asarray(mesh.vertices)
    return torch.from_numpy(v[tri.flatten()].reshape(len(tri), 3, 3)).to(device).float()


def _force_cost(force_norm, clamp_max):
    return -(force_norm * torch.nn.functional.softmin(force_norm, dim=1)).clamp(max=clamp_max).sum(dim=1)


def _sdf_normal(points, faces, faces_deflate):
    """SDF distance / sign / blended normal (:182-187): the normal averages the deflated and the
    true mesh's signed normals (flips inside the object)."""
    _, sign1, n1, _ = compute_sdf(points, faces_deflate)
    dist, sign2, n2, _ = compute_sdf(points, faces)
    n = 0.5 * sign1.unsqueeze(1) * n1 + 0.5 * sign2.unsqueeze(1) * n2
    return dist, n / n.norm(dim=1).unsqueeze(1)


class _Best:
    """Best-iterate tracking of the four loops without host syncs."""

    def __init__(self, l0_dtype, E, T, device, **params):
        self.value = torch.full((E,), float("inf"), dtype=l0_dtype, device=device)
        self.margin = torch.zeros(E, T, dtype=torch.float64, device=device)
        self.normal = None
        self.params = {k: v.detach().clone() for k, v in params.items()}

    @torch.no_grad()
    def update(self, l, margin, normal, **params):
        flag = l < self.value
        anyf = flag.any()
        self.margin = torch.where(anyf, margin, self.margin)
        self.normal = normal if self.normal is None else torch.where(anyf, normal, self.normal)
        self.value = torch.where(flag, l.to(self.value.dtype), self.value)
        for k, v in params.items():
            m = flag.view((-1,) + (1,) * (v.dim() - 1))
            self.params[k] = torch.where(m, v.detach(), self.params[k])

    def flag(self):
        return (self.margin > 0.0).all()


def _noise(tape, s):
    return None if tape is None else tape[s]


class _FusedLoop:
    """Device state of a fused Kin / SDF loop: the two prepared meshes, cdx_kin_cost's outputs (margin / normal
    in two alternating slots), the optimiser moments, the best iterate and the cdx_kin_step buffers.  Per
    iteration the loop is three TorchSDF queries, cdx_kin_cost and cdx_kin_step (optimiser, best iterate,
    clamps and — Kin — the next fingertips' FK): no autograd graph, no host sync."""

    def __init__(self, E, T, pose, target, comp, faces, faces_deflate, dev):
        f32 = dict(dtype=torch.float32, device=dev)
        self.mesh, self.mesh_def = PreparedMesh(faces), PreparedMesh(faces_deflate)
        self.ws_tips, self.ws_tgt = QueryWorkspace(), QueryWorkspace()
        # the batched launch's schedule (heaviest point groups of the last iteration first; CDX_SDF_SCHED=0: none)
        self.sched = BatchSchedule()
        self.iteration = 0
        self.hist = None
        # iterations per point sort: 16 (A/B with the batched launch's schedule, profiles/r05ba_config4_resort_sched_ab.jsonl:
        # 4 / 8 / 16 / never = 0.327 / 0.316 / 0.316 / 0.311 ms around the mesh, 0.461 / 0.445 / 0.442 / 0.469 far)
        self.resort = max(1, int(os.environ.get("CDX_SDF_RESORT", "16")))
        # the three queries' outputs (dist, sign, normals, clst), and the two side streams the second and third
        # query run on beside the first (CDX_SDF_CONCURRENT=0: all three on the caller's stream)
        self.q_out = [(torch.empty(E * T, **f32), torch.empty(E * T, dtype=torch.int32, device=dev),
                       torch.empty(E * T, 3, **f32), torch.empty(E * T, 3, **f32)) for _ in range(3)]
        # 3 (default): the three queries in one launch (cdx_sdf_query_batch); 1: on three streams; 2: the targets' on
        # a side stream only; 0: one after the other (A/B switch CDX_SDF_CONCURRENT)
        self.concurrent = int(os.environ.get("CDX_SDF_CONCURRENT", "3"))
        if self.concurrent == 3 and not (self.mesh.kind == N.SDF_MESH_CULLED and self.mesh_def.kind == N.SDF_MESH_CULLED):
            self.concurrent = 1  # (a mesh with NaN-capable faces: the batch launch has no exact path)
        if self.concurrent in (1, 2):
            self.side = [torch.cuda.Stream(device=dev) for _ in range(2)]
            self.ev = [torch.cuda.Event() for _ in range(4)]
        self.pose, self.target, self.comp = pose, target, comp
        self.loss = torch.empty(E, dtype=torch.float64, device=dev)
        self.margin = [torch.zeros(E, T, dtype=torch.float64, device=dev) for _ in range(2)]
        self.normal = [torch.zeros(E * T, 3, **f32) for _ in range(2)]
        self.g = [torch.empty_like(pose), torch.empty_like(target), torch.empty_like(comp)]
        self.m = [torch.zeros_like(pose), torch.zeros_like(target), torch.zeros_like(comp)]
        self.v = [torch.zeros_like(pose), torch.zeros_like(target), torch.zeros_like(comp)]
        self.opt_value = torch.full((E,), float("inf"), **f32)
        self.opt_margin = torch.zeros(E, T, dtype=torch.float64, device=dev)
        self.opt_normal = torch.zeros(E * T, 3, **f32)
        self.opt = [pose.clone(), target.clone(), comp.clone()]
        self.any = torch.zeros(3, dtype=torch.int32, device=dev)
        self.tips = torch.empty(E * T, 3, **f32)
        b = N.CdxKinOptBuffers()
        for name, t in (("pose", pose), ("target", target), ("comp", comp), ("g_pose", self.g[0]),
                        ("g_target", self.g[1]), ("g_comp", self.g[2]), ("m_pose", self.m[0]), ("v_pose", self.v[0]),
                        ("m_target", self.m[1]), ("v_target", self.v[1]), ("m_comp", self.m[2]), ("v_comp", self.v[2]),
                        ("loss", self.loss), ("opt_value", self.opt_value), ("opt_margin", self.opt_margin),
                        ("opt_normal", self.opt_normal), ("opt_pose", self.opt[0]), ("opt_target", self.opt[1]),
                        ("opt_comp", self.opt[2]), ("any", self.any)):
            setattr(b, name, N.ptr(t))
        for i in range(2):
            b.margin[i], b.normal[i] = N.ptr(self.margin[i]), N.ptr(self.normal[i])
        self.buffers = b

    def queries(self, tips, target):
        """The iteration's three TorchSDF calls (:186-188).  The fingertips are sorted once for both meshes, and the
        fingertips' and targets' orders are re-sorted only every ``resort`` iterations: a query's results do not
        depend on the order its points are walked in (each point's winner is exact), only the culling's speed does,
        and the points move little between iterations."""
        fresh = self.iteration % self.resort == 0
        self.iteration += 1
        tgt = target.view(-1, 3)
        o = self.q_out
        if self.concurrent == 3:
            # one launch: each culled kernel's tail (a few point groups far from the mesh) leaves most of the chip idle,
            # which the other queries' groups fill — no side stream, no event
            if fresh:
                self.ws_tips.sort(tips)
                self.ws_tgt.sort(tgt)
            query_batch([(self.mesh_def, tips, self.ws_tips, o[0]), (self.mesh, tips, self.ws_tips, o[1]),
                         (self.mesh, tgt, self.ws_tgt, o[2])], schedule=self.sched)
        elif not self.concurrent:
            if fresh:  # (sorted explicitly: a query on a mesh with NaN-capable faces neither sorts nor walks)
                self.ws_tips.sort(tips)
                self.ws_tgt.sort(tgt)
            self.mesh_def.query(tips, workspace=self.ws_tips, reuse_order=True, out=o[0])
            self.mesh.query(tips, workspace=self.ws_tips, reuse_order=True, out=o[1])
            self.mesh.query(tgt, workspace=self.ws_tgt, reuse_order=True, out=o[2])
        else:
            # The three queries are independent: each culled kernel's tail (a few point groups far from the mesh)
            # leaves most of the chip idle, which the others fill.  The targets are sorted (when fresh) and queried
            # on side stream 2, the fingertips sorted on the caller's stream and queried against the full mesh on
            # side stream 1 and against the deflated mesh on the caller's, which waits for both before cdx_kin_cost.
            main = torch.cuda.current_stream(tips.device)
            ev_start, ev_tips, ev_full, ev_tgt = self.ev
            ev_start.record(main)
            s1, s2 = self.side
            s2.wait_event(ev_start)
            with torch.cuda.stream(s2):
                if fresh:
                    self.ws_tgt.sort(tgt)
                self.mesh.query(tgt, workspace=self.ws_tgt, reuse_order=True, out=o[2])
            ev_tgt.record(s2)
            if fresh:
                self.ws_tips.sort(tips)
            if self.concurrent == 1:
                ev_tips.record(main)
                s1.wait_event(ev_tips)
                with torch.cuda.stream(s1):
                    self.mesh.query(tips, workspace=self.ws_tips, reuse_order=True, out=o[1])
                ev_full.record(s1)
            self.mesh_def.query(tips, workspace=self.ws_tips, reuse_order=True, out=o[0])
            if self.concurrent == 1:
                main.wait_event(ev_full)
            else:  # (A/B: the full mesh's fingertip query on the caller's stream too)
                self.mesh.query(tips, workspace=self.ws_tips, reuse_order=True, out=o[1])
            main.wait_event(ev_tgt)
        return o[0][1], o[0][2], o[1][0], o[1][1], o[1][2], o[1][3], o[2][0], o[2][1], o[2][3]

    def loss_slot(self, s, iters):
        """Iteration s's loss vector: a row of a per-call [iters, E] history (the per-iteration sums are taken in one
        reduction after the loop, not one per iteration), or the single buffer when the history would pass 1 GiB."""
        E = self.loss.shape[0]
        if s == 0:
            self.hist = (torch.empty(iters, E, dtype=torch.float64, device=self.loss.device)
                         if iters * E * 8 <= (1 << 30) else None)
        row = self.hist[s] if self.hist is not None else self.loss
        self.buffers.loss = N.ptr(row)
        return row

    def loss_sums(self, history):
        """Append the loop's per-iteration loss sums (device scalars) to ``history``."""
        if getattr(self, "hist", None) is not None:
            history.extend(self.hist.sum(dim=1).unbind(0))

    def best(self):
        return self.opt[0], self.opt[2], self.opt[1], (self.opt_margin > 0.0).all()


class KinGraspOptimizer:
    """Joint-space optimiser on the TorchSDF mesh distance (optimize_pregrasp.py:121-227)."""

    def __init__(self, robot_urdf, ee_link_names, ee_link_offsets=EE_OFFSETS, palm_offset=(-0.01, 0.015, 0.12),
                 num_iters=1000, optimize_target=False, ref_q=None, mass=0.1, com=(0.0, 0.0, 0.0), gravity=True,
                 uncertainty=0.0, device="cuda", seed=0):
        """``seed``: key of the fused loop's on-device Kabsch noise (used when no ``kabsch_noise`` tape is given);
        iteration k of this optimiser's n-th fused call draws with key seed + (iterations before it) + k + 1."""
        self.device = torch.device(device)
        self._seed = int(seed)
        self.loop_events = None  # optional (start, end) CUDA events around a fused loop's iterations
        self.ref_q = torch.tensor(list(ref_q)).to(self.device)
        self.robot_model = DifferentiableRobotModel(robot_urdf, device=device)
        self.num_iters = num_iters
        self.ee_link_names = list(ee_link_names)
        self.ee_link_offsets = ee_link_offsets
        self.palm_offset = torch.tensor(palm_offset).to(self.device)
        self.optimize_target = optimize_target
        self.gravity, self.mass, self.com = gravity, mass, list(com)

    def forward_kinematics(self, joint_angles):
        """[E·T, 3] fingertips: FK (recursive=True, :148) + palm offset."""
        tips = self.robot_model.compute_forward_kinematics(joint_angles, self.ee_link_names,
                                                          offsets=self.ee_link_offsets, recursive=True)[0]
        return (tips.view(-1, 3) + self.palm_offset).view(-1, 3)

    def optimize(self, joint_angles, target_pose, compliance, friction_mu, object_mesh, verbose=True,
                 kabsch_noise=None, trace_rows=False, fused=True):
        """``trace_rows``: also keep every iteration's per-candidate loss in ``loss_rows`` (device).
        ``fused`` (default): per iteration the three TorchSDF queries on prepared meshes, ONE cost-and-backward
        kernel (cdx_kin_cost: force_eq_reward, the six cost terms and the backward through them, TorchSDF and
        the FK chain) and ONE step kernel (cdx_kin_step: Adam, the best iterate, the next fingertips' FK) — no
        autograd graph, no host sync; ``fused=False``: the same loop through the autograd drop-ins
        (compute_sdf, force_eq_reward, the FK module), torch tensor ops and torch.optim.Adam, as the reference
        writes it."""
        self.loss_history = []
        self.loss_rows = []
        faces = _face_vertices(object_mesh, self.device)
        object_mesh.scale(0.9, center=[0, 0, 0])
        faces_deflate = _face_vertices(object_mesh, self.device)
        E, T = target_pose.shape[0], target_pose.shape[1]
        lrs = (2e-3, 1e-5, 0.2) if self.optimize_target else (1e-2, 0.0, 0.2)  # q, target, compliance (:168-176)
        if fused:
            return self._optimize_fused(joint_angles, target_pose, compliance, friction_mu, faces, faces_deflate, lrs,
                                        verbose, kabsch_noise, trace_rows)
        joint_angles = joint_angles.clone().requires_grad_(True)
        compliance = compliance.clone().requires_grad_(True)
        if self.optimize_target:
            target_pose = target_pose.clone().requires_grad_(True)
            optim = torch.optim.Adam([{"params": joint_angles, "lr": lrs[0]}, {"params": target_pose, "lr": lrs[1]},
                                      {"params": compliance, "lr": lrs[2]}])
        else:
            optim = torch.optim.Adam([{"params": joint_angles, "lr": lrs[0]}, {"params": compliance, "lr": lrs[2]}])
        best = _Best(torch.float32, E, T, self.device, q=joint_angles, comp=compliance, target=target_pose)
        for s in range(self.num_iters):
            optim.zero_grad()
            all_tip = self.forward_kinematics(joint_angles)
            dist, normal = _sdf_normal(all_tip, faces, faces_deflate)
            tar_dist, tar_sign, _, _ = compute_sdf(target_pose.reshape(-1, 3), faces)
            reward, margin, force_norm = force_eq_reward(
                all_tip.view(target_pose.shape), target_pose, compliance, friction_mu, normal.view(target_pose.shape),
                mass=self.mass, COM=self.com, gravity=10.0 if self.gravity else None, kabsch_noise=_noise(kabsch_noise, s))
            c = -reward * 5.0
            center_cost = (all_tip.view(target_pose.shape).mean(dim=1) - target_pose.mean(dim=1)).norm(dim=1) * 10.0
            ref_cost = (joint_angles - self.ref_q).norm(dim=1) * 10.0
            dist_cost = 1000 * torch.sqrt(dist).view(E, T).sum(dim=1)
            # the reference multiplies tar_sign [E·T] into the [E, T] view (:211), which only broadcasts
            # for E = 1; the [E, T] sign is what that line means and what it computes at E = 1
            tar_dist_cost = 10 * (tar_sign.view(E, T) * torch.sqrt(tar_dist).view(E, T)).sum(dim=1)
            l = c + dist_cost + tar_dist_cost + center_cost + _force_cost(force_norm, 1.0) + ref_cost
            l.sum().backward()
            self.loss_history.append(l.detach().sum())  # device scalar, no sync
            if trace_rows:
                self.loss_rows.append(l.detach().clone())
            if verbose:
                print("Loss:", float(l.sum()), compliance)
            best.update(l, margin, normal, q=joint_angles, comp=compliance, target=target_pose)
            optim.step()
        if verbose:
            print(best.margin, best.normal)
        self.best_loss = best.value
        return best.params["q"], best.params["comp"], best.params["target"], best.flag()

    def _optimize_fused(self, joint_angles, target_pose, compliance, friction_mu, faces, faces_deflate, lrs, verbose,
                        kabsch_noise, trace_rows):
        lib = N.load()
        dev = self.device
        E, T = target_pose.shape[0], target_pose.shape[1]
        q, tgt, comp = (x.detach().clone().contiguous() for x in (joint_angles, target_pose, compliance))
        if any(x.dtype != torch.float32 for x in (q, tgt, comp)):
            raise ValueError("KinGraspOptimizer: joint angles, targets and compliances must be float32 (the "
                             "reference's dtype on this path)")
        chain = self.robot_model._descriptor(self.ee_link_names, self.ee_link_offsets)
        prm = N.CdxKinParams()
        prm.fe = force_eq_descriptor(T, friction_mu, self.mass, 10.0 if self.gravity else None, 2.0, self.com)
        for i, v in enumerate(self.ref_q.float().tolist()):
            prm.ref_q[i] = v
        cfg = N.CdxKinOpt()
        cfg.rule, cfg.clamp_box = 0, 0
        cfg.lr[0], cfg.lr[1], cfg.lr[2] = lrs
        cfg.beta1, cfg.beta2, cfg.eps = 0.9, 0.999, 1e-8  # torch.optim.Adam defaults (:171)
        off = self.palm_offset.float().cpu().tolist()
        for i in range(3):
            cfg.palm_offset[i] = off[i]
        st = _FusedLoop(E, T, q, tgt, comp, faces, faces_deflate, dev)
        st.buffers.tips = N.ptr(st.tips)
        # (A/B: "0" cdx_kin_cost + cdx_kin_step; "alt" the two forms alternating, even iterations two launches — a
        # test hook: the one-launch iterations then find the FK-walk cache one step stale and must walk)
        fused_step = os.environ.get("CDX_KIN_FUSED_STEP", "1")
        one_launch = fused_step != "0"
        nb = int(lib.cdx_kin_fk_state_bytes(E, T))
        if one_launch and nb and os.environ.get("CDX_KIN_FK_CACHE", "1") != "0":  # (A/B: every iteration walks)
            # the step's FK walk kept for the next iteration's FK backward (any contents: the kernel tags what it wrote)
            st.fk_state = torch.full((nb // 4,), -1, dtype=torch.int32, device=dev)
            st.buffers.fk_state = N.ptr(st.fk_state)
        stream = N.stream_ptr(dev)
        N.check(lib.cdx_fk_forward(chain, N.ptr(q), E, N.ptr(st.tips), None, stream), "cdx_fk_forward")
        st.tips.add_(self.palm_offset.float())  # FK + palm offset (:148); later iterations: cdx_kin_step
        if self.loop_events:
            self.loop_events[0].record()
        for s in range(self.num_iters):
            nz = _noise(kabsch_noise, s)
            nz = None if nz is None else nz.detach().to(device=dev, dtype=torch.float64).contiguous()
            self._seed += 1
            loss = st.loss_slot(s, self.num_iters)
            qr = [N.ptr(t) for t in st.queries(st.tips, tgt)]
            if not verbose and one_launch and not (fused_step == "alt" and s % 2 == 0):
                # cost, backward and step in one launch (cdx_kin_iteration)
                N.check(lib.cdx_kin_iteration(chain, prm, cfg, st.buffers, E, T, *qr, N.ptr(nz), self._seed, s, stream),
                        "cdx_kin_iteration")
            else:  # two launches (verbose: the compliances printed before the step, as the reference prints them)
                N.check(lib.cdx_kin_cost(chain, prm, E, N.ptr(q), N.ptr(st.tips), N.ptr(tgt), N.ptr(comp), *qr,
                                         N.ptr(nz), self._seed, N.ptr(loss), N.ptr(st.margin[s & 1]),
                                         N.ptr(st.normal[s & 1]), N.ptr(st.g[0]), N.ptr(st.g[1]), N.ptr(st.g[2]), None,
                                         stream), "cdx_kin_cost")
                if verbose:
                    print("Loss:", float(loss.sum()), comp)
                N.check(lib.cdx_kin_step(chain, cfg, st.buffers, E, T, s, 0, stream), "cdx_kin_step")
            if st.hist is None:
                self.loss_history.append(loss.sum())  # device scalar, no sync
            if trace_rows:
                self.loss_rows.append(loss.clone())
        N.check(lib.cdx_kin_step(chain, cfg, st.buffers, E, T, self.num_iters, 1, stream), "cdx_kin_step")
        st.loss_sums(self.loss_history)
        if self.loop_events:
            self.loop_events[1].record()
        if verbose:
            print(st.opt_margin, st.opt_normal)
        self.best_loss = st.opt_value
        # the last iteration's per-candidate loss and fingertips (device, no copy; the reference prints the
        # non-finite case at :212-213)
        self.last_loss, self.last_tips = (loss if self.num_iters else None), st.tips
        self.last_params = (q, tgt, comp)  # the parameters after the last step (device, updated in place)
        # (trace_rows: the loop's device state too — moments, best iterate — for state-injection checks)
        self.last_loop = st if trace_rows else None
        return st.best()


class SDFGraspOptimizer:
    """Fingertip-space optimiser on the TorchSDF mesh distance (optimize_pregrasp.py:229-320)."""

    def __init__(self, tip_bounding_box, num_iters=2000, optimize_target=False, mass=0.1, com=(0.0, 0.0, 0.0),
                 gravity=True, uncertainty=0.0, device="cuda", seed=0):
        """``seed``: key of the fused loop's on-device Kabsch noise (as KinGraspOptimizer's)."""
        self.device = torch.device(device)
        self._seed = int(seed)
        self.loop_events = None  # optional (start, end) CUDA events around a fused loop's iterations
        self.tip_bounding_box = [torch.tensor(tip_bounding_box[0]).to(self.device).view(-1, 3),
                                 torch.tensor(tip_bounding_box[1]).to(self.device).view(-1, 3)]
        self.num_iters = num_iters
        self.optimize_target = optimize_target
        self.mass, self.com, self.gravity = mass, list(com), gravity

    def optimize(self, tip_pose, target_pose, compliance, friction_mu, object_mesh, verbose=True, kabsch_noise=None,
                 trace_rows=False, fused=True):
        """``trace_rows``: also keep every iteration's per-candidate loss in ``loss_rows`` (device).
        ``fused`` (default): per iteration the three TorchSDF queries on prepared meshes, ONE cost-and-backward
        kernel (cdx_kin_cost without a chain) and ONE step kernel (cdx_kin_step: RMSprop, the best iterate, the
        box clamps); ``fused=False``: the autograd loop with torch.optim.RMSprop."""
        self.loss_history = []
        self.loss_rows = []
        faces = _face_vertices(object_mesh, self.device)
        object_mesh.scale(0.9, center=[0, 0, 0])
        faces_deflate = _face_vertices(object_mesh, self.device)
        E, T = tip_pose.shape[0], tip_pose.shape[1]
        lrs = (1e-3, 1e-3 if self.optimize_target else 0.0, 0.2)  # tips, target, compliance (:250-259)
        if fused:
            return self._optimize_fused(tip_pose, target_pose, compliance, friction_mu, faces, faces_deflate, lrs,
                                        verbose, kabsch_noise, trace_rows)
        tip_pose = tip_pose.clone().requires_grad_(True)
        compliance = compliance.clone().requires_grad_(True)
        if self.optimize_target:
            target_pose = target_pose.clone().requires_grad_(True)
            optim = torch.optim.RMSprop([{"params": tip_pose, "lr": lrs[0]}, {"params": target_pose, "lr": lrs[1]},
                                         {"params": compliance, "lr": lrs[2]}])
        else:
            optim = torch.optim.RMSprop([{"params": tip_pose, "lr": lrs[0]}, {"params": compliance, "lr": lrs[2]}])
        best = _Best(torch.float32, E, T, self.device, tip=tip_pose, comp=compliance, target=target_pose)
        for s in range(self.num_iters):
            optim.zero_grad()
            all_tip = tip_pose.view(-1, 3)
            dist, normal = _sdf_normal(all_tip, faces, faces_deflate)
            tar_dist, tar_sign, _, _ = compute_sdf(target_pose.reshape(-1, 3), faces)
            reward, margin, force_norm = force_eq_reward(
                tip_pose, target_pose, compliance, friction_mu, normal.view(tip_pose.shape), mass=self.mass,
                COM=self.com, gravity=10.0 if self.gravity else None, kabsch_noise=_noise(kabsch_noise, s))
            c = -reward * 5.0
            center_cost = (tip_pose.mean(dim=1) - target_pose.mean(dim=1)).norm(dim=1) * 10.0
            dist_cost = 1000 * torch.sqrt(dist).view(E, T).sum(dim=1)
            tar_dist_cost = 10 * (torch.sqrt(tar_dist).view(E, T) * tar_sign.view(E, T)).sum(dim=1)  # see :297
            l = c + dist_cost + tar_dist_cost + center_cost + _force_cost(force_norm, 1.0)
            l.sum().backward()
            self.loss_history.append(l.detach().sum())  # device scalar, no sync
            if trace_rows:
                self.loss_rows.append(l.detach().clone())
            if verbose:
                print("Loss:", float(l.sum()), float(dist_cost.sum()), float(tar_dist_cost.sum()))
            best.update(l, margin, normal, tip=tip_pose, comp=compliance, target=target_pose)
            optim.step()
            with torch.no_grad():  # bounding-box constraints (:312-314)
                tip_pose.clamp_(min=self.tip_bounding_box[0], max=self.tip_bounding_box[1])
                target_pose.clamp_(min=self.tip_bounding_box[0], max=self.tip_bounding_box[1])
        if verbose:
            print(best.margin, best.normal)
        self.best_loss = best.value
        return best.params["tip"], best.params["comp"], best.params["target"], best.flag()

    def _optimize_fused(self, tip_pose, target_pose, compliance, friction_mu, faces, faces_deflate, lrs, verbose,
                        kabsch_noise, trace_rows):
        lib = N.load()
        dev = self.device
        E, T = tip_pose.shape[0], tip_pose.shape[1]
        tips, tgt, comp = (x.detach().clone().contiguous() for x in (tip_pose, target_pose, compliance))
        if any(x.dtype != torch.float32 for x in (tips, tgt, comp)):
            raise ValueError("SDFGraspOptimizer: tip poses, targets and compliances must be float32 (TorchSDF's path)")
        prm = N.CdxKinParams()
        prm.fe = force_eq_descriptor(T, friction_mu, self.mass, 10.0 if self.gravity else None, 2.0, self.com)
        cfg = N.CdxKinOpt()
        cfg.rule, cfg.clamp_box = 1, 1
        cfg.lr[0], cfg.lr[1], cfg.lr[2] = lrs
        cfg.alpha, cfg.eps = 0.99, 1e-8  # torch.optim.RMSprop defaults (:253)
        lb = self.tip_bounding_box[0].float().expand(T, 3).reshape(-1).cpu().tolist()
        ub = self.tip_bounding_box[1].float().expand(T, 3).reshape(-1).cpu().tolist()
        for i in range(3 * T):
            cfg.box_lb[i], cfg.box_ub[i] = lb[i], ub[i]
        st = _FusedLoop(E, T, tips, tgt, comp, faces, faces_deflate, dev)
        stream = N.stream_ptr(dev)
        one_launch = os.environ.get("CDX_KIN_FUSED_STEP", "1") != "0"  # (A/B: cdx_kin_cost + cdx_kin_step)
        if self.loop_events:
            self.loop_events[0].record()
        for s in range(self.num_iters):
            nz = _noise(kabsch_noise, s)
            nz = None if nz is None else nz.detach().to(device=dev, dtype=torch.float64).contiguous()
            self._seed += 1
            pts = tips.view(-1, 3)
            loss = st.loss_slot(s, self.num_iters)
            qr = [N.ptr(t) for t in st.queries(pts, tgt)]
            if not verbose and one_launch:  # cost, backward and step in one launch (cdx_kin_iteration)
                N.check(lib.cdx_kin_iteration(None, prm, cfg, st.buffers, E, T, *qr, N.ptr(nz), self._seed, s, stream),
                        "cdx_kin_iteration")
            else:
                N.check(lib.cdx_kin_cost(None, prm, E, None, N.ptr(pts), N.ptr(tgt), N.ptr(comp), *qr, N.ptr(nz),
                                         self._seed, N.ptr(loss), N.ptr(st.margin[s & 1]), N.ptr(st.normal[s & 1]),
                                         None, N.ptr(st.g[1]), N.ptr(st.g[2]), N.ptr(st.g[0]), stream), "cdx_kin_cost")
                if verbose:
                    print("Loss:", float(loss.sum()))
                N.check(lib.cdx_kin_step(None, cfg, st.buffers, E, T, s, 0, stream), "cdx_kin_step")
            if st.hist is None:
                self.loss_history.append(loss.sum())  # device scalar, no sync
            if trace_rows:
                self.loss_rows.append(loss.clone())
        N.check(lib.cdx_kin_step(None, cfg, st.buffers, E, T, self.num_iters, 1, stream), "cdx_kin_step")
        st.loss_sums(self.loss_history)
        if self.loop_events:
            self.loop_events[1].record()
        if verbose:
            print(st.opt_margin, st.opt_normal)
        self.best_loss = st.opt_value
        return st.best()


class GPISGraspOptimizer:
    """Fingertip-space optimiser on the GPIS distance and variance (optimize_pregrasp.py:322-406)."""

    def __init__(self, tip_bounding_box, num_iters=2000, optimize_target=False, mass=0.1, com=(0.0, 0.0, 0.0),
                 gravity=True, uncertainty=20.0, device="cuda"):
        self.device = torch.device(device)
        self.tip_bounding_box = [torch.tensor(tip_bounding_box[0]).to(self.device).view(-1, 3),
                                 torch.tensor(tip_bounding_box[1]).to(self.device).view(-1, 3)]
        self.num_iters = num_iters
        self.optimize_target = optimize_target
        self.mass, self.com, self.gravity, self.uncertainty = mass, list(com), gravity, uncertainty

    def optimize(self, tip_pose, target_pose, compliance, friction_mu, gpis, verbose=True, kabsch_noise=None):
        tip_pose = tip_pose.clone().requires_grad_(True)
        self.loss_history = []
        compliance = compliance.clone().requires_grad_(True)
        if self.optimize_target:
            target_pose = target_pose.clone().requires_grad_(True)
            optim = torch.optim.RMSprop([{"params": tip_pose, "lr": 1e-3}, {"params": target_pose, "lr": 1e-3},
                                         {"params": compliance, "lr": 0.2}])
        else:
            optim = torch.optim.RMSprop([{"params": tip_pose, "lr": 1e-3}, {"params": compliance, "lr": 0.2}])
        E, T = tip_pose.shape[0], tip_pose.shape[1]
        best = _Best(torch.float64, E, T, self.device, tip=tip_pose, comp=compliance, target=target_pose)
        for s in range(self.num_iters):
            optim.zero_grad()
            all_tip = tip_pose.view(-1, 3)
            dist, var = gpis.pred(all_tip)
            tar_dist, _ = gpis.pred(target_pose.reshape(-1, 3))
            normal = gpis.compute_normal(all_tip)
            reward, margin, force_norm = force_eq_reward(
                tip_pose, target_pose, compliance, friction_mu, normal.view(tip_pose.shape), mass=self.mass,
                COM=self.com, gravity=10.0 if self.gravity else None, kabsch_noise=_noise(kabsch_noise, s))
            c = -reward * 25.0
            center_cost = (tip_pose.mean(dim=1) - target_pose.mean(dim=1)).norm(dim=1) * 10.0
            dist_cost = 1000 * torch.abs(dist).view(E, T).sum(dim=1)
            tar_dist_cost = 10 * tar_dist.view(E, T).sum(dim=1)
            variance_cost = self.uncertainty * var.view(E, T).sum(dim=1)
            l = c + dist_cost + tar_dist_cost + center_cost + _force_cost(force_norm, 1.0) + variance_cost
            l.sum().backward()
            self.loss_history.append(l.detach().sum())  # device scalar, no sync
            if verbose:
                print("Loss:", float(l.sum()), float(dist_cost.sum()), float(variance_cost.sum()))
            best.update(l, margin, normal, tip=tip_pose, comp=compliance, target=target_pose)
            optim.step()
            with torch.no_grad():  # (:399-401)
                tip_pose.clamp_(min=self.tip_bounding_box[0], max=self.tip_bounding_box[1])
                compliance.clamp_(min=40.0)
        if verbose:
            print(best.margin, best.normal)
        self.best_loss = best.value
        return best.params["tip"], best.params["comp"], best.params["target"], best.flag()


class KinGPISGraspOptimizer:
    """Joint-space optimiser on the GPIS distance and log-variance (optimize_pregrasp.py:408-511)."""

    def __init__(self, robot_urdf, ee_link_names, ee_link_offsets=EE_OFFSETS, palm_offset=WRIST_OFFSET, num_iters=1000,
                 optimize_target=False, ref_q=None, tip_bounding_box=(FINGERTIP_LB, FINGERTIP_UB), mass=0.1,
                 com=(0.0, 0.0, 0.0), gravity=True, uncertainty=10.0, device="cuda"):
        self.device = torch.device(device)
        self.ref_q = torch.tensor(list(ref_q)).to(self.device)
        self.robot_model = DifferentiableRobotModel(robot_urdf, device=device)
        self.num_iters = num_iters
        self.ee_link_names = list(ee_link_names)
        self.ee_link_offsets = ee_link_offsets
        self.palm_offset = torch.tensor(np.asarray(palm_offset)).double().to(self.device)
        self.optimize_target = optimize_target
        self.tip_bounding_box = [torch.tensor(tip_bounding_box[0]).to(self.device).view(-1, 3),
                                 torch.tensor(tip_bounding_box[1]).to(self.device).view(-1, 3)]
        self.mass, self.com, self.gravity, self.uncertainty = mass, list(com), gravity, uncertainty

    def forward_kinematics(self, joint_angles):
        tips = self.robot_model.compute_forward_kinematics(joint_angles, self.ee_link_names,
                                                          offsets=self.ee_link_offsets, recursive=True)[0]
        return (tips.view(-1, 3) + self.palm_offset).view(-1, 3)

    def optimize(self, joint_angles, target_pose, compliance, friction_mu, gpis, verbose=True, kabsch_noise=None):
        joint_angles = joint_angles.clone().requires_grad_(True)
        self.loss_history = []
        compliance = compliance.clone().requires_grad_(True)
        if self.optimize_target:
            target_pose = target_pose.clone().requires_grad_(True)
            optim = torch.optim.RMSprop([{"params": joint_angles, "lr": 2e-3}, {"params": target_pose, "lr": 1e-3},
                                         {"params": compliance, "lr": 0.2}])
        else:
            optim = torch.optim.RMSprop([{"params": joint_angles, "lr": 1e-2}, {"params": compliance, "lr": 0.2}])
        E, T = target_pose.shape[0], target_pose.shape[1]
        best = _Best(torch.float64, E, T, self.device, q=joint_angles, comp=compliance, target=target_pose)
        for s in range(self.num_iters):
            optim.zero_grad()
            all_tip = self.forward_kinematics(joint_angles)
            dist, var = gpis.pred(all_tip)
            tar_dist, _ = gpis.pred(target_pose.reshape(-1, 3))
            normal = gpis.compute_normal(all_tip)
            reward, margin, force_norm = force_eq_reward(
                all_tip.view(target_pose.shape), target_pose, compliance, friction_mu, normal.view(target_pose.shape),
                mass=self.mass, COM=self.com, gravity=10.0 if self.gravity else None, kabsch_noise=_noise(kabsch_noise, s))
            c = -reward * 5.0
            center_cost = (all_tip.view(target_pose.shape).mean(dim=1) - target_pose.mean(dim=1)).norm(dim=1) * 10.0
            ref_cost = (joint_angles - self.ref_q).norm(dim=1) * 20.0
            variance_cost = self.uncertainty * torch.log(100 * var).view(E, T)
            dist_cost = 1000 * torch.abs(dist).view(E, T).sum(dim=1)
            tar_dist_cost = 10 * tar_dist.view(E, T).sum(dim=1)
            l = (c + dist_cost + tar_dist_cost + center_cost + _force_cost(force_norm, 1.0) + ref_cost +
                 variance_cost.max(dim=1)[0])
            l.sum().backward()
            self.loss_history.append(l.detach().sum())  # device scalar, no sync
            if verbose:
                print("Loss:", float(l.sum()), variance_cost.detach())
            best.update(l, margin, normal, q=joint_angles, comp=compliance, target=target_pose)
            optim.step()
            with torch.no_grad():  # (:503-505)
                compliance.clamp_(min=40.0)
                target_pose.clamp_(min=self.tip_bounding_box[0], max=self.tip_bounding_box[1])
        if verbose:
            print(best.margin, best.normal)
        self.best_loss = best.value
        return best.params["q"], best.params["comp"], best.params["target"], best.flag()
