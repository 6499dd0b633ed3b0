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

import numpy as np
import torch

from . import _native as N
from .force_eq import force_eq_descriptor, force_eq_reward
from .optimizer import EE_OFFSETS, FINGERTIP_LB, FINGERTIP_UB, WRIST_OFFSET
from .robot_model import DifferentiableRobotModel
from .torchsdf import _forward as _sdf_query
from .torchsdf import compute_sdf


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


class KinGraspOptimizer:
    """Joint-space optimiser on the TorchSDF mesh distance (optimize_pregrasp.py:121-227)."""

    def __init__(self, robot_urdf, ee_link_names, ee_link_offsets=EE_OFFSETS, palm_offset=(-0.01, 0.015, 0.12),
                 num_iters=1000, optimize_target=False, ref_q=None, mass=0.1, com=(0.0, 0.0, 0.0), gravity=True,
                 uncertainty=0.0, device="cuda"):
        self.device = torch.device(device)
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
        ``fused`` (default): per iteration one FK launch, the three TorchSDF queries on cached prepared
        meshes and ONE cost-and-backward kernel (cdx_kin_cost: force_eq_reward, the six cost terms and the
        backward through them, TorchSDF and the FK chain) writing the parameters' gradients — no autograd
        graph; ``fused=False``: the same loop through the autograd drop-ins (compute_sdf, force_eq_reward,
        the FK module) and torch tensor ops, as the reference writes it."""
        self.loss_history = []
        self.loss_rows = []
        joint_angles = joint_angles.clone().requires_grad_(True)
        compliance = compliance.clone().requires_grad_(True)
        faces = _face_vertices(object_mesh, self.device)
        object_mesh.scale(0.9, center=[0, 0, 0])
        faces_deflate = _face_vertices(object_mesh, self.device)
        # the fused loop also takes torch's single-kernel Adam (same update rule; one launch per step instead
        # of the foreach path's ≈ 21 — profiles/r04d_config4_kin_iteration_split.json)
        afused = dict(fused=True) if fused and self.device.type == "cuda" else {}
        if self.optimize_target:
            target_pose = target_pose.clone().requires_grad_(True)
            optim = torch.optim.Adam([{"params": joint_angles, "lr": 2e-3}, {"params": target_pose, "lr": 1e-5},
                                      {"params": compliance, "lr": 0.2}], **afused)
        else:
            optim = torch.optim.Adam([{"params": joint_angles, "lr": 1e-2}, {"params": compliance, "lr": 0.2}],
                                     **afused)
        E, T = target_pose.shape[0], target_pose.shape[1]
        best = _Best(torch.float32, E, T, self.device, q=joint_angles, comp=compliance, target=target_pose)
        if fused:
            return self._optimize_fused(joint_angles, target_pose, compliance, friction_mu, faces, faces_deflate,
                                        optim, best, verbose, kabsch_noise, trace_rows)
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

    def _optimize_fused(self, joint_angles, target_pose, compliance, friction_mu, faces, faces_deflate, optim, best,
                        verbose, kabsch_noise, trace_rows):
        lib = N.load()
        dev = self.device
        E, T = target_pose.shape[0], target_pose.shape[1]
        chain = self.robot_model._descriptor(self.ee_link_names, self.ee_link_offsets)
        D = chain.n_dofs
        prm = N.CdxKinParams()
        prm.fe = force_eq_descriptor(T, friction_mu, self.mass, 10.0 if self.gravity else None, 2.0, self.com)
        for i, v in enumerate(self.ref_q.float().tolist()):
            prm.ref_q[i] = v
        f32 = dict(dtype=torch.float32, device=dev)
        tips = torch.empty(E * T, 3, **f32)
        loss = torch.empty(E, dtype=torch.float64, device=dev)
        margin = torch.empty(E, T, dtype=torch.float64, device=dev)
        normal = torch.empty(E * T, 3, **f32)
        g_q, g_target, g_comp = torch.empty(E, D, **f32), torch.empty(E, T, 3, **f32), torch.empty(E, T, **f32)
        offset = self.palm_offset.float()
        stream = N.stream_ptr(dev)
        for s in range(self.num_iters):
            q = joint_angles.detach()
            if not q.is_contiguous() or q.dtype != torch.float32:
                raise ValueError("KinGraspOptimizer: joint angles must be a contiguous float32 tensor")
            N.check(lib.cdx_fk_forward(chain, N.ptr(q), E, N.ptr(tips), None, stream), "cdx_fk_forward")
            tips.add_(offset)  # FK + palm offset (:148)
            tgt = target_pose.detach().reshape(-1, 3).contiguous()
            _, sign1, n1, _, _ = _sdf_query(tips, faces_deflate, False)
            dist, sign2, n2, clst, _ = _sdf_query(tips, faces, False)
            tdist, tsign, _, tclst, _ = _sdf_query(tgt, faces, False)
            nz = _noise(kabsch_noise, s)
            nz = None if nz is None else nz.detach().to(device=dev, dtype=torch.float64).contiguous()
            comp = compliance.detach().contiguous()
            N.check(lib.cdx_kin_cost(chain, prm, E, N.ptr(q), N.ptr(tips), N.ptr(tgt), N.ptr(comp), N.ptr(sign1),
                                     N.ptr(n1), N.ptr(dist), N.ptr(sign2), N.ptr(n2), N.ptr(clst), N.ptr(tdist),
                                     N.ptr(tsign), N.ptr(tclst), N.ptr(nz), next(_kin_seeds), N.ptr(loss), N.ptr(margin),
                                     N.ptr(normal), N.ptr(g_q), N.ptr(g_target), N.ptr(g_comp), None, stream),
                    "cdx_kin_cost")
            joint_angles.grad = g_q.clone()
            compliance.grad = g_comp.clone()
            if self.optimize_target:
                target_pose.grad = g_target.clone()
            self.loss_history.append(loss.sum())  # device scalar, no sync
            if trace_rows:
                self.loss_rows.append(loss.clone())
            if verbose:
                print("Loss:", float(loss.sum()), compliance)
            best.update(loss, margin, normal.clone(), q=joint_angles, comp=compliance, target=target_pose)
            optim.step()
        if verbose:
            print(best.margin, best.normal)
        self.best_loss = best.value
        return best.params["q"], best.params["comp"], best.params["target"], best.flag()


_kin_seeds = __import__("itertools").count(0x6B1)


class SDFGraspOptimizer:
    """Fingertip-space optimiser on the TorchSDF mesh distance (optimize_pregrasp.py:229-320)."""

    def __init__(self, tip_bounding_box, num_iters=2000, optimize_target=False, mass=0.1, com=(0.0, 0.0, 0.0),
                 gravity=True, uncertainty=0.0, device="cuda"):
        self.device = torch.device(device)
        self.tip_bounding_box = [torch.tensor(tip_bounding_box[0]).to(self.device).view(-1, 3),
                                 torch.tensor(tip_bounding_box[1]).to(self.device).view(-1, 3)]
        self.num_iters = num_iters
        self.optimize_target = optimize_target
        self.mass, self.com, self.gravity = mass, list(com), gravity

    def optimize(self, tip_pose, target_pose, compliance, friction_mu, object_mesh, verbose=True, kabsch_noise=None,
                 trace_rows=False, fused=True):
        """``trace_rows``: also keep every iteration's per-candidate loss in ``loss_rows`` (device).
        ``fused`` (default): per iteration the three TorchSDF queries on cached prepared meshes and ONE
        cost-and-backward kernel (cdx_kin_cost without a chain); ``fused=False``: the autograd loop."""
        tip_pose = tip_pose.clone().requires_grad_(True)
        self.loss_history = []
        self.loss_rows = []
        compliance = compliance.clone().requires_grad_(True)
        faces = _face_vertices(object_mesh, self.device)
        object_mesh.scale(0.9, center=[0, 0, 0])
        faces_deflate = _face_vertices(object_mesh, self.device)
        if self.optimize_target:
            target_pose = target_pose.clone().requires_grad_(True)
            optim = torch.optim.RMSprop([{"params": tip_pose, "lr": 1e-3}, {"params": target_pose, "lr": 1e-3},
                                         {"params": compliance, "lr": 0.2}])
        else:
            optim = torch.optim.RMSprop([{"params": tip_pose, "lr": 1e-3}, {"params": compliance, "lr": 0.2}])
        E, T = tip_pose.shape[0], tip_pose.shape[1]
        best = _Best(torch.float32, E, T, self.device, tip=tip_pose, comp=compliance, target=target_pose)
        if fused:
            return self._optimize_fused(tip_pose, target_pose, compliance, friction_mu, faces, faces_deflate, optim,
                                        best, verbose, kabsch_noise, trace_rows)
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

    def _optimize_fused(self, tip_pose, target_pose, compliance, friction_mu, faces, faces_deflate, optim, best,
                        verbose, kabsch_noise, trace_rows):
        lib = N.load()
        dev = self.device
        E, T = tip_pose.shape[0], tip_pose.shape[1]
        prm = N.CdxKinParams()
        prm.fe = force_eq_descriptor(T, friction_mu, self.mass, 10.0 if self.gravity else None, 2.0, self.com)
        f32 = dict(dtype=torch.float32, device=dev)
        loss = torch.empty(E, dtype=torch.float64, device=dev)
        margin = torch.empty(E, T, dtype=torch.float64, device=dev)
        normal = torch.empty(E * T, 3, **f32)
        g_tip, g_target, g_comp = torch.empty(E, T, 3, **f32), torch.empty(E, T, 3, **f32), torch.empty(E, T, **f32)
        stream = N.stream_ptr(dev)
        for s in range(self.num_iters):
            tips = tip_pose.detach().reshape(-1, 3).contiguous()
            tgt = target_pose.detach().reshape(-1, 3).contiguous()
            if tips.dtype != torch.float32 or tgt.dtype != torch.float32:
                raise ValueError("SDFGraspOptimizer: tip and target poses must be float32 (TorchSDF's path)")
            _, sign1, n1, _, _ = _sdf_query(tips, faces_deflate, False)
            dist, sign2, n2, clst, _ = _sdf_query(tips, faces, False)
            tdist, tsign, _, tclst, _ = _sdf_query(tgt, faces, False)
            nz = _noise(kabsch_noise, s)
            nz = None if nz is None else nz.detach().to(device=dev, dtype=torch.float64).contiguous()
            comp = compliance.detach().contiguous()
            N.check(lib.cdx_kin_cost(None, prm, E, None, N.ptr(tips), N.ptr(tgt), N.ptr(comp), N.ptr(sign1), N.ptr(n1),
                                     N.ptr(dist), N.ptr(sign2), N.ptr(n2), N.ptr(clst), N.ptr(tdist), N.ptr(tsign),
                                     N.ptr(tclst), N.ptr(nz), next(_kin_seeds), N.ptr(loss), N.ptr(margin),
                                     N.ptr(normal), None, N.ptr(g_target), N.ptr(g_comp), N.ptr(g_tip), stream),
                    "cdx_kin_cost")
            tip_pose.grad = g_tip.clone()
            compliance.grad = g_comp.clone()
            if self.optimize_target:
                target_pose.grad = g_target.clone()
            self.loss_history.append(loss.sum())  # device scalar, no sync
            if trace_rows:
                self.loss_rows.append(loss.clone())
            if verbose:
                print("Loss:", float(loss.sum()))
            best.update(loss, margin, normal.clone(), tip=tip_pose, comp=compliance, target=target_pose)
            optim.step()
            with torch.no_grad():  # bounding-box constraints (:312-314)
                tip_pose.clamp_(min=self.tip_bounding_box[0], max=self.tip_bounding_box[1])
                target_pose.clamp_(min=self.tip_bounding_box[0], max=self.tip_bounding_box[1])
        if verbose:
            print(best.margin, best.normal)
        self.best_loss = best.value
        return best.params["tip"], best.params["comp"], best.params["target"], best.flag()


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
