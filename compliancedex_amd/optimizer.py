"""Drop-in for ``ProbabilisticGraspOptimizer`` (optimize_pregrasp.py:614-839) on MI355X.

``closure`` is ONE native call (cdx_closure: FK → GPIS queries → fused cost + analytic
backward) that writes the five parameter gradients straight into ``.grad``; ``optimize``
keeps the reference's loop (Adam, best-iterate tracking after step 20, compliance and
target clamps).  Module constants mirror optimize_pregrasp.py:13-30.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _native as N
from .problem import build_problem
from .robot_model import DifferentiableRobotModel

EE_OFFSETS = [[0.0, -0.04, 0.015], [0.0, -0.04, 0.015], [0.0, -0.04, 0.015], [0.0, -0.05, -0.015]]
WRIST_OFFSET = np.array([[-0.06, 0.0, 0.05, 0.0, 0.0, 0.0],
                         [-0.04, 0.03, 0.05, 0.0, 0.0, -np.pi / 4],
                         [-0.01, 0.0, 0.05, 0.0, 0.0, np.pi / 4],
                         [0.1, 0.06, 0.03, -np.pi / 2, np.pi / 2, 0.0],
                         [-0.0, -0.06, 0.05, 0.0, 0.0, np.pi / 2],
                         [0.02, -0.04, 0.05, 0.0, 0.0, 3 * np.pi / 4]])
z_margin = 0.2
FINGERTIP_LB = [-0.2, -0.2, 0.015, -0.2, -0.2, 0.015, -0.2, -0.2, 0.015, -0.2, -0.2, 0.015]
FINGERTIP_UB = [0.2, 0.2, z_margin, 0.2, 0.2, z_margin, 0.2, 0.2, z_margin, 0.2, 0.2, z_margin]


def euler_angles_to_matrix(euler_angles, convention="XYZ"):
    """Rx·Ry·Rz for convention XYZ (math_utils.py:68-123); other conventions as the reference."""
    if euler_angles.dim() == 0 or euler_angles.shape[-1] != 3:
        raise ValueError("Invalid input euler angles.")
    if len(convention) != 3 or convention[1] in (convention[0], convention[2]) or any(c not in "XYZ" for c in convention):
        raise ValueError(f"Invalid convention {convention}.")

    def rot(axis, t):
        c, s = torch.cos(t), torch.sin(t)
        one, zero = torch.ones_like(t), torch.zeros_like(t)
        m = {"X": (one, zero, zero, zero, c, -s, zero, s, c),
             "Y": (c, zero, s, zero, one, zero, -s, zero, c),
             "Z": (c, -s, zero, s, c, zero, zero, zero, one)}[axis]
        return torch.stack(m, -1).reshape(t.shape + (3, 3))

    mats = [rot(c, e) for c, e in zip(convention, torch.unbind(euler_angles, -1))]
    return torch.matmul(torch.matmul(mats[0], mats[1]), mats[2])


class ProbabilisticGraspOptimizer:
    def __init__(self, robot_urdf, ee_link_names, ee_link_offsets=EE_OFFSETS, palm_offset=WRIST_OFFSET,
                 num_iters=1000, optimize_target=False, ref_q=None, tip_bounding_box=(FINGERTIP_LB, FINGERTIP_UB),
                 pregrasp_coefficients=((0.8, 0.8, 0.8, 0.8),) * 3, pregrasp_weights=(0.1, 0.8, 0.1),
                 anchor_link_names=None, anchor_link_offsets=None, collision_pairs=None,
                 collision_pair_threshold=0.02, mass=0.1, com=(0.0, 0.0, 0.0), gravity=True, uncertainty=20.0,
                 optimize_palm=False, device="cuda", seed=0):
        self.device = torch.device(device)
        self.ref_q = torch.tensor(list(ref_q)).to(self.device)  # float32 (:634)
        self.robot_model = DifferentiableRobotModel(robot_urdf, device=device)
        self.num_iters = num_iters
        self.ee_link_names = list(ee_link_names)
        self.ee_link_offsets = [list(map(float, o)) for o in ee_link_offsets] if ee_link_offsets is not None else None
        self.palm_offset = torch.from_numpy(np.asarray(palm_offset, dtype=np.float64)).to(self.device)
        self.optimize_target = optimize_target
        self.optimize_palm = optimize_palm
        self.tip_bounding_box = [torch.tensor(tip_bounding_box[0]).to(self.device).view(-1, 3),
                                 torch.tensor(tip_bounding_box[1]).to(self.device).view(-1, 3)]
        self.pregrasp_coefficients = torch.tensor([list(r) for r in pregrasp_coefficients]).to(self.device)
        self.pregrasp_weights = torch.tensor(list(pregrasp_weights)).double().to(self.device)
        self.anchor_link_names = anchor_link_names
        self.anchor_link_offsets = anchor_link_offsets
        if collision_pairs is not None:
            cp = torch.tensor(collision_pairs).long().to(self.device)
            self.collision_pair_left, self.collision_pair_right = cp[:, 0], cp[:, 1]
        self.collision_pair_threshold = collision_pair_threshold
        self.mass, self.com, self.gravity, self.uncertainty = mass, list(com), gravity, uncertainty
        self._chain_desc = self.robot_model._descriptor(self.ee_link_names, self.ee_link_offsets)
        self._problem = self._problem_state = self._problem_key = None
        self._ws = None
        self._seed = int(seed)
        self.optim = None

    # ------------------------------------------------------------------ FK
    def forward_kinematics(self, joint_angles, palm_poses=None):
        """World fingertips R(euler XYZ)·tip + palm_pos, [E, 4, 3] f64 (:657-669)."""
        if palm_poses is None:
            palm_poses = self.palm_offset
        tips = self.robot_model.compute_forward_kinematics(joint_angles.float(), self.ee_link_names,
                                                           offsets=self.ee_link_offsets)[0].double().view(-1, 4, 3)
        R = euler_angles_to_matrix(palm_poses[:, 3:], convention="XYZ")
        return torch.bmm(R, tips.transpose(1, 2)).transpose(1, 2) + palm_poses[:, :3].unsqueeze(1)

    def compute_collision_loss(self, joint_angles, palm_poses=None):
        """Pairwise / floor / palm proximity penalty (:671-701; disabled in the reference closure, :765)."""
        if palm_poses is None:
            palm_poses = self.palm_offset
        anchor = self.robot_model.compute_forward_kinematics(joint_angles.float(), self.anchor_link_names,
                                                             offsets=self.anchor_link_offsets)[0].double()
        anchor = anchor.view(-1, len(self.anchor_link_names), 3)
        R = euler_angles_to_matrix(palm_poses[:, 3:], convention="XYZ")
        anchor = torch.bmm(R, anchor.transpose(1, 2)).transpose(1, 2) + palm_poses[:, :3].unsqueeze(1)
        dist = torch.norm(anchor[:, self.collision_pair_left] - anchor[:, self.collision_pair_right], dim=2)
        inv = torch.where(dist < self.collision_pair_threshold, 1.0 / dist, torch.zeros_like(dist))
        cost = inv.sum(dim=1)
        z = anchor[:, :, 2]
        cost = cost + torch.where(z < 0.02, 0.1 / z, torch.zeros_like(z)).sum(dim=1)
        if self.optimize_palm:
            pz = palm_poses[:, 2]
            cost = cost + torch.where(pz < 0.02, 1 / pz, torch.zeros_like(pz))
        return cost

    # --------------------------------------------------------------- closure
    def problem(self, gpis, friction_mu):
        """cdx_problem for this GPIS state and friction (rebuilt only when either changes)."""
        st = gpis.native_state()
        key = (id(st), float(friction_mu))
        if self._problem_key != key:
            self._problem = build_problem(self._chain_desc, st.desc, ref_q=self.ref_q.tolist(),
                                          coeffs=self.pregrasp_coefficients.tolist(),
                                          weights=self.pregrasp_weights.tolist(), mu=friction_mu, mass=self.mass,
                                          com=self.com, gravity=self.gravity, uncertainty=self.uncertainty,
                                          optimize_palm=self.optimize_palm)
            self._problem_state = st  # the descriptor points into this state's buffers
            self._problem_key = key
        return self._problem

    def closure(self, joint_angles, compliance, target_pose, palm_poses, palm_oris, friction_mu, gpis, num_envs,
                kabsch_noise=None):
        """One cost+grad eval for all candidates (:741-769).  ``kabsch_noise`` [K·E, 3, 3]
        replays the reference's ``rand_like(H)`` draw; by default it is drawn on device."""
        if self.optim is not None:
            self.optim.zero_grad()
        lib = N.load()
        p = self.problem(gpis, friction_mu)
        E = int(num_envs)
        dev = joint_angles.device
        f64 = dict(dtype=torch.float64, device=dev)
        q = joint_angles.detach().to(torch.float64).contiguous()
        comp = compliance.detach().to(torch.float64).contiguous()
        target = target_pose.detach().to(torch.float64).contiguous()
        pp = palm_poses.detach().to(torch.float64).contiguous()
        po = palm_oris.detach().to(torch.float64).contiguous()
        T, D = p.chain.n_tips, p.chain.n_dofs
        if q.shape != (E, D) or comp.shape != (E, T) or target.shape != (E, T, 3) or pp.shape != (E, 3) or po.shape != (E, 3):
            raise ValueError("closure input shapes do not match num_envs / the hand")
        need = lib.cdx_closure_workspace(p, E)
        if self._ws is None or self._ws.numel() < need:
            self._ws = torch.empty(need, dtype=torch.uint8, device=dev)
        total_loss = torch.empty(E, **f64)
        total_margin = torch.empty(E, T, **f64)
        pre = torch.empty(E, T, 3, **f64)
        g = [torch.empty(E, D, **f64), torch.empty(E, T, **f64), torch.empty(E, T, 3, **f64), torch.empty(E, 3, **f64),
             torch.empty(E, 3, **f64)]
        noise = None
        if kabsch_noise is not None:
            noise = kabsch_noise.to(**f64).contiguous()
            if noise.numel() != p.n_levels * E * 9:
                raise ValueError("kabsch_noise must be [K*E, 3, 3]")
        flip = torch.empty(p.n_levels * E, dtype=torch.int32, device=dev)
        self._seed += 1
        N.check(lib.cdx_closure(p, E, N.ptr(q), N.ptr(comp), N.ptr(target), N.ptr(pp), N.ptr(po), N.ptr(noise),
                                self._seed, N.ptr(self._ws), N.ptr(total_loss), N.ptr(total_margin), N.ptr(pre),
                                *[N.ptr(t) for t in g], N.ptr(flip), N.stream_ptr(dev)), "cdx_closure")
        for param, grad in zip((joint_angles, compliance, target_pose, palm_poses, palm_oris), g):
            if param.requires_grad and param.is_leaf:
                grad = grad.to(param.dtype)
                param.grad = grad if param.grad is None else param.grad + grad
        self.pregrasp_tip_pose = pre
        self.total_loss = total_loss
        self.total_margin = total_margin
        self.kabsch_flip = flip  # det(V·Uᵀ) < 0 mask per (level, candidate) (:64)
        return total_loss.sum()

    # -------------------------------------------------------------- optimize
    def optimize(self, init_joint_angles, target_pose, compliance, friction_mu, gpis, verbose=True,
                 noise_tape=None):
        """The reference's Adam loop (:771-839).  ``noise_tape``: optional per-iteration
        Kabsch noise tensors (parity replay)."""
        joint_angles = init_joint_angles.clone().requires_grad_(True)
        compliance = compliance.clone().requires_grad_(True)
        params_list = [{"params": joint_angles, "lr": 1e-3}, {"params": compliance, "lr": 0.2}]
        if self.optimize_target:
            target_pose = target_pose.clone().requires_grad_(True)
            params_list.append({"params": target_pose, "lr": 2e-3})
        palm_poses = self.palm_offset[:, :3].clone().requires_grad_(self.optimize_palm)
        palm_oris = self.palm_offset[:, 3:].clone().requires_grad_(self.optimize_palm)
        if self.optimize_palm:
            params_list.append({"params": palm_poses, "lr": 1e-4})
            params_list.append({"params": palm_oris, "lr": 1e-4})
        self.optim = torch.optim.Adam(params_list)
        num_envs = init_joint_angles.shape[0]
        opt_joint_angle = init_joint_angles.clone()
        opt_compliance = compliance.clone()
        opt_target_pose = target_pose.clone()
        opt_value = torch.inf * torch.ones(num_envs, dtype=torch.float64, device=joint_angles.device)
        opt_margin = torch.zeros(num_envs, 4, dtype=torch.float64, device=joint_angles.device)
        opt_palm_poses = self.palm_offset.clone()
        for s in range(self.num_iters):
            noise = noise_tape[s] if noise_tape is not None else None
            self.closure(joint_angles, compliance, target_pose, palm_poses, palm_oris, friction_mu, gpis, num_envs,
                         kabsch_noise=noise)
            with torch.no_grad():
                update_flag = self.total_loss < opt_value
                if s > 20:  # (:823) — masked updates need no host sync
                    opt_value = torch.where(update_flag, self.total_loss, opt_value)
                    m1 = update_flag.unsqueeze(1)
                    opt_margin = torch.where(m1, self.total_margin, opt_margin)
                    opt_joint_angle = torch.where(m1, joint_angles.to(opt_joint_angle.dtype), opt_joint_angle)
                    opt_target_pose = torch.where(update_flag.view(-1, 1, 1), target_pose, opt_target_pose)
                    opt_compliance = torch.where(m1, compliance, opt_compliance)
                    opt_palm_poses = torch.where(m1, torch.hstack([palm_poses, palm_oris]), opt_palm_poses)
            self.optim.step()
            with torch.no_grad():
                compliance.clamp_(min=80.0)
                target_pose.clamp_(min=self.tip_bounding_box[0], max=self.tip_bounding_box[1])
        self.best_loss = opt_value
        if verbose:
            print("Margin:", opt_margin)
        return opt_joint_angle, opt_compliance, opt_target_pose, opt_palm_poses, opt_margin
