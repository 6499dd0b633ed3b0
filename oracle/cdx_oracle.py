"""ORACLE — test infrastructure only.  CPU (torch) restatement of the ComplianceDex
probabilistic-pregrasp hot path, used to CHECK the HIP path; never shipped, never a
fallback.  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import it.

Pinning: every function here is checked against golden vectors produced by running
the reference itself (``tests/golden/make_golden.py``; ``tests/test_oracle_golden.py``).

The restatement keeps the reference's dtype mix: FK in float32, GPIS
and cost in float64, float32-rounded constants (cos_mu, pregrasp coefficients, ref_q,
dummy-gravity spring), and its gradient artifacts (detached quaternion scale,
detached normals, injected Kabsch noise).  It keeps the reference's computational
structure too (LU solve per call, the full M×M posterior covariance whose diagonal is
taken), because the same code is timed as the CPU baseline.
"""
from __future__ import annotations

import math

import torch

F32, F64 = torch.float32, torch.float64


# ----------------------------------------------------------------------------- GPIS
def tps_kernel(xa, xb, R):
    """Thin-plate-spline kernel 2r³ − 3Rr² + R³ on cdist (gpis.py:21-26)."""
    r = torch.cdist(xa, xb)
    return 2 * r ** 3 - 3 * R * r ** 2 + R ** 3


def rbf_kernel(xa, xb, sigma):
    """Exponentiated quadratic exp(−r²/2σ²) (gpis.py:16-19)."""
    return torch.exp(-0.5 * torch.cdist(xa, xb) ** 2 / sigma ** 2)


class OracleGPIS:
    """GP implicit surface state + queries (gpis.py:4-168)."""

    def __init__(self, X1, y1, E11, R, bias, kernel="tps", sigma=0.08):
        self.X1 = torch.as_tensor(X1, dtype=F64)
        self.y1 = torch.as_tensor(y1, dtype=F64).reshape(-1, 1)
        self.E11 = torch.as_tensor(E11, dtype=F64)
        self.R = torch.as_tensor(R, dtype=F64)
        self.bias = torch.as_tensor(bias).double()
        self.kernel = kernel
        self.sigma = sigma

    @classmethod
    def fit(cls, X1, y, noise, bias=1.0, kernel="tps", sigma=0.08):
        """E11 = K(X1,X1) + diag(noise²), R = max pairwise distance (gpis.py:33-40)."""
        X1 = torch.as_tensor(X1, dtype=F64)
        y = torch.as_tensor(y, dtype=F64).reshape(-1, 1)
        noise = torch.as_tensor(noise, dtype=F64)
        R = torch.max(torch.cdist(X1, X1))
        self = cls(X1, y - bias, torch.zeros(len(X1), len(X1), dtype=F64), R, bias, kernel, sigma)
        self.E11 = self.k(X1, X1) + (noise ** 2) * torch.eye(len(X1), dtype=F64)
        return self

    @classmethod
    def from_npz(cls, path):
        import numpy as np
        d = np.load(path)
        return cls(d["X1"], d["y1"], d["E11"], d["R"], d["bias"])

    def k(self, xa, xb):
        if self.kernel == "tps":
            return tps_kernel(xa, xb, self.R)
        if self.kernel == "rbf":
            return rbf_kernel(xa, xb, self.sigma)
        return 0.3 * rbf_kernel(xa, xb, self.sigma) + 0.7 * tps_kernel(xa, xb, self.R)

    def pred(self, X2):
        """(mean, sqrt|diag Σ|) with the reference's solve + full M×M E22 (gpis.py:43-59)."""
        shape = list(X2.shape[:-1])
        X2 = X2.reshape(-1, 3)
        E12 = self.k(self.X1, X2)
        solved = torch.linalg.solve(self.E11, E12).T
        mu = solved @ self.y1 + self.bias
        E2 = self.k(X2, X2) - solved @ E12
        return mu.reshape(shape), torch.sqrt(torch.abs(torch.diagonal(E2))).reshape(shape)

    def compute_normal(self, X2, index=None):
        """∇mean/(‖∇mean‖+1e-8) with the inverse-based weight, detached (gpis.py:63-87)."""
        shape = X2.shape
        idx = torch.arange(len(self.X1)) if index is None else torch.as_tensor(index)
        with torch.enable_grad():
            X = X2.detach().reshape(-1, 3).clone().requires_grad_(True)
            E12 = self.k(self.X1, X)
            weight = (torch.inverse(self.E11) @ self.y1)[idx]
            (E12[idx].T @ weight).sum().backward()
            g = X.grad
        n = g / (torch.norm(g, dim=1, keepdim=True) + 1e-8)
        if index is None:
            return n.view(shape)
        return n.view(shape), weight.sum()

    def compute_multinormals(self, X2, num_normal_samples):
        """Normals of nested inducing-point subsets (gpis.py:89-111): fractions linspace(0.8, 1)
        of the leading points, all points, then ranges from ``int(1 − fraction)`` (= 0: the
        reference's index quirk makes the trailing half full sets)."""
        n = len(self.X1)
        frac = torch.linspace(0.8, 1, num_normal_samples // 2)
        idx = [list(range(int(frac[i] * n))) for i in range(num_normal_samples // 2)]
        idx.append(list(range(n)))
        idx += [list(range(int(1 - frac[-i - 1]), n)) for i in range(num_normal_samples // 2)]
        normals, weights = [], []
        for ix in idx:
            nrm, w = self.compute_normal(X2, ix)
            normals.append(nrm)
            weights.append(w)
        weights = torch.hstack(weights)
        return torch.stack(normals, dim=1), weights / weights.sum()


# ------------------------------------------------------------------------------- FK
def _axis_rot(axis, ang):
    """x_rot / y_rot / z_rot in float32 (spatial_vector_algebra.py:14-53)."""
    B = ang.shape[0]
    c, s = torch.cos(ang), torch.sin(ang)
    one, zero = torch.ones(B, dtype=ang.dtype), torch.zeros(B, dtype=ang.dtype)
    if axis == 0:
        rows = (one, zero, zero, zero, c, -s, zero, s, c)
    elif axis == 1:
        rows = (c, zero, s, zero, one, zero, -s, zero, c)
    else:
        rows = (c, -s, zero, s, c, zero, zero, zero, one)
    return torch.stack(rows, -1).view(B, 3, 3)


def fixed_rotation(rpy):
    """(Rz(yaw)·Ry(pitch))·Rx(roll) in float32 (rigid_body.py:138-144)."""
    r = torch.as_tensor(rpy, dtype=F32).view(3, 1)
    return (_axis_rot(2, r[2]) @ _axis_rot(1, r[1])) @ _axis_rot(0, r[0])


class OracleChain:
    """Batched rigid-body tree FK, non-recursive form (robot_model.py:140-196, 224-264).

    ``bodies``: list of dicts {name, parent (index or -1), xyz, rpy, axis (3 floats),
    joint ('fixed' or other)} in URDF link order.  Controlled joints get DOF indices in
    that order (robot_model.py:115-131)."""

    def __init__(self, bodies):
        self.bodies = bodies
        self.index = {b["name"]: i for i, b in enumerate(bodies)}
        self.F = [fixed_rotation(b["rpy"])[0] for b in bodies]
        self.t = [torch.as_tensor(b["xyz"], dtype=F32) for b in bodies]
        self.dof = []
        n = 0
        for b in bodies:
            if b["joint"] != "fixed" and b["parent"] >= 0:
                self.dof.append(n)
                n += 1
            else:
                self.dof.append(-1)
        self.n_dofs = n

    def _joint_rot(self, i, q):
        """Axis handling of rigid_body.py:149-155: only unit ±x/±y/±z are recognised;
        anything else falls to z with sign(axis_z)."""
        ax = torch.as_tensor(self.bodies[i]["axis"], dtype=F32)
        if torch.abs(ax[0]) == 1:
            return _axis_rot(0, torch.sign(ax[0]) * q)
        if torch.abs(ax[1]) == 1:
            return _axis_rot(1, torch.sign(ax[1]) * q)
        return _axis_rot(2, torch.sign(ax[2]) * q)

    def world_poses(self, q):
        B = q.shape[0]
        rot = [None] * len(self.bodies)
        trans = [None] * len(self.bodies)
        rot[0] = torch.eye(3, dtype=F32).expand(B, 3, 3)
        trans[0] = torch.zeros(B, 3, dtype=F32)
        for i in range(1, len(self.bodies)):
            p = self.bodies[i]["parent"]
            if self.dof[i] >= 0:
                Rj = self.F[i].expand(B, 3, 3) @ self._joint_rot(i, q[:, self.dof[i]])
            else:
                Rj = self.F[i].expand(B, 3, 3)
            rot[i] = rot[p] @ Rj
            trans[i] = (rot[p] @ self.t[i].view(1, 3, 1)).squeeze(2) + trans[p]
        return rot, trans

    @staticmethod
    def quaternion(R):
        """xyzw quaternion with the reference's branch and its DETACHED scale
        (spatial_vector_algebra.py:108-136: ``math.sqrt`` on a tensor leaves autograd)."""
        B = R.shape[0]
        M33 = 1.0
        t = R[:, 0, 0] + R[:, 1, 1] + R[:, 2, 2] + M33
        out = []
        for n in range(B):
            Mn = R[n]
            if t[n] > M33:
                tn = t[n]
                qn = torch.stack([Mn[2, 1] - Mn[1, 2], Mn[0, 2] - Mn[2, 0], Mn[1, 0] - Mn[0, 1], tn])
            else:
                i, j, k = 0, 1, 2
                if Mn[1, 1] > Mn[0, 0]:
                    i, j, k = 1, 2, 0
                if Mn[2, 2] > Mn[i, i]:
                    i, j, k = 2, 0, 1
                tn = Mn[i, i] - (Mn[j, j] + Mn[k, k]) + M33
                comp = [None] * 4
                comp[i] = tn
                comp[j] = Mn[i, j] + Mn[j, i]
                comp[k] = Mn[k, i] + Mn[i, k]
                comp[3] = Mn[k, j] - Mn[j, k]
                qn = torch.stack(comp)
            scale = 0.5 / math.sqrt(float(tn.detach()) * M33)
            out.append(qn * torch.tensor(scale, dtype=F32))
        return torch.stack(out)

    @staticmethod
    def quat_rotate(q, v):
        """v(2w²−1) + 2w(q×v) + 2q(q·v) (se3_so3_util.py:240-250)."""
        w = q[:, 3:4]
        qv = q[:, :3]
        return v * (2.0 * w ** 2 - 1.0) + torch.cross(qv, v, dim=-1) * w * 2.0 + \
            qv * (qv * v).sum(-1, keepdim=True) * 2.0

    def forward_kinematics(self, q, link_names, offsets=None):
        """→ (pos [B, 3L] f32, quat [B, 4L] f32) (robot_model.py:248-264)."""
        q = q.to(F32)
        rot, trans = self.world_poses(q)
        poses, quats = [], []
        for li, name in enumerate(link_names):
            i = self.index[name]
            pos = trans[i]
            quat = self.quaternion(rot[i])
            if offsets is not None:
                off = torch.as_tensor(offsets[li], dtype=F32).view(1, 3).expand(q.shape[0], 3)
                pos = pos + self.quat_rotate(quat, off)
            poses.append(pos)
            quats.append(quat)
        return torch.cat(poses, 1), torch.cat(quats, 1)


def euler_xyz(angles):
    """R = Rx(a)·Ry(b)·Rz(c) (math_utils.py:68-123, convention "XYZ")."""
    a, b, c = angles.unbind(-1)

    def rot(axis, t):
        co, si = torch.cos(t), torch.sin(t)
        one, zero = torch.ones_like(t), torch.zeros_like(t)
        if axis == "X":
            m = (one, zero, zero, zero, co, -si, zero, si, co)
        elif axis == "Y":
            m = (co, zero, si, zero, one, zero, -si, zero, co)
        else:
            m = (co, -si, zero, si, co, zero, zero, zero, one)
        return torch.stack(m, -1).reshape(t.shape + (3, 3))

    return torch.matmul(torch.matmul(rot("X", a), rot("Y", b)), rot("Z", c))


# ----------------------------------------------------------------------------- cost
def kabsch(S1, S2, w, noise):
    """Weighted Kabsch with injected SVD noise (optimize_pregrasp.py:49-69).
    ``noise`` is the tensor the reference draws with ``rand_like(H)`` at :61."""
    w = w.unsqueeze(2)
    c1 = S1.mean(dim=1, keepdim=True)
    c2 = S2.mean(dim=1, keepdim=True)
    H = (w * (S1 - c1)).transpose(1, 2) @ (w * (S2 - c2))
    Hn = H + 1e-6 * noise
    # A non-finite batch element (a diverged candidate) comes out NaN on the reference's CUDA path and the loop goes
    # on (its `isnan` print, :212-213); torch's CPU LAPACK path raises instead, so only the finite rows are factored
    fin = torch.isfinite(Hn).flatten(1).all(dim=1)
    if bool(fin.all()):
        U, _, Vh = torch.linalg.svd(Hn)
    else:
        U = torch.full_like(Hn, float("nan"))
        Vh = torch.full_like(Hn, float("nan"))
        if bool(fin.any()):
            U[fin], _, Vh[fin] = torch.linalg.svd(Hn[fin])
    V = Vh.mH
    flip = torch.linalg.det(V @ U.transpose(1, 2)) < 0.0
    sign = torch.ones(S1.shape[0], 3, 3, dtype=F32)
    sign[flip, :, -1] = -1.0
    R = (V * sign) @ U.transpose(1, 2)
    t = (w * (S2 - (R @ S1.transpose(1, 2)).transpose(1, 2))).sum(dim=1) / w.sum(dim=1)
    return R, t, flip


def cos_friction(mu):
    """sqrt(1/(1+mu²)) evaluated the reference's way: torch.tensor(mu) then default-dtype
    (float32) division (optimize_pregrasp.py:111,707)."""
    return torch.sqrt(1 / (1 + torch.tensor(mu) ** 2))


def force_eq_reward(tip, target, comp, mu, normal, noise, mass=0.1, gravity=10.0, M=2.0, COM=(0.0, 0.0, 0.0)):
    """Equilibrium of the compliant grasp + friction-cone margin (optimize_pregrasp.py:73-118)."""
    B = tip.shape[0]
    if gravity is None:
        R, t, flip = kabsch(tip, target, comp, noise)
        return _eq_terms(tip, target, comp, mu, normal, R, t) + (flip,)
    dummy_tip = torch.zeros(B, 1, 3, dtype=F32)
    dummy_tip[:, 0, :] = torch.tensor(COM, dtype=F64)
    dummy_target = torch.zeros(B, 1, 3, dtype=F32)
    dummy_target[:, 0, 2] = -M
    dummy_comp = gravity * mass / M * torch.ones(B, 1, dtype=F32)
    R, t, flip = kabsch(torch.cat([tip, dummy_tip], 1), torch.cat([target, dummy_target], 1),
                        torch.cat([comp, dummy_comp], 1), noise)
    return _eq_terms(tip, target, comp, mu, normal, R, t) + (flip,)


def _eq_terms(tip, target, comp, mu, normal, R, t):
    tip_eq = (R @ tip.transpose(1, 2)).transpose(1, 2) + t.unsqueeze(1)
    diff = tip_eq - target
    force = comp.unsqueeze(2) * (-diff)
    direction = diff / diff.norm(dim=2).unsqueeze(2)
    normal_eq = (R @ normal.transpose(1, 2)).transpose(1, 2)
    ang = (direction * normal_eq).sum(-1)
    margin = (ang - cos_friction(mu)).clamp(min=-0.9999)
    reward = (0.2 * torch.log(ang + 1) + 0.8 * torch.log(margin + 1)).sum(dim=1)
    return reward, margin, force.norm(dim=2)


def contact_margin(tip, target, normal, mu):
    """Unclamped contact-margin reward (optimize_pregrasp.py:703-710)."""
    d = tip - target
    d = d / d.norm(dim=2, keepdim=True)
    ang = (d * normal).sum(-1)
    m = ang - cos_friction(mu)
    return (0.1 * torch.log(ang + 1) + 0.9 * torch.log(m + 1)).sum(dim=1)


PREGRASP_COEFFS = [[0.8] * 4] * 3
PREGRASP_WEIGHTS = [0.1, 0.8, 0.1]


class OracleProblem:
    """The prob-mode optimiser's fixed data (optimize_pregrasp.py:614-655)."""

    def __init__(self, chain, ee_links, ee_offsets, ref_q, gpis, mu=1, mass=0.1, com=(0.0, 0.0, 0.0),
                 gravity=True, uncertainty=20.0, optimize_palm=True,
                 coeffs=PREGRASP_COEFFS, weights=PREGRASP_WEIGHTS):
        self.chain = chain
        self.ee_links = list(ee_links)
        self.ee_offsets = [list(map(float, o)) for o in ee_offsets]
        self.ref_q = torch.tensor(list(map(float, ref_q)))          # float32 (:634)
        self.gpis = gpis
        self.mu = mu
        self.mass, self.com, self.gravity = mass, tuple(com), gravity
        self.uncertainty = uncertainty
        self.optimize_palm = optimize_palm
        self.coeffs = torch.tensor(coeffs)                            # float32 (:644)
        self.weights = torch.tensor(weights).double()                 # float64 (:645)

    def forward_kinematics(self, q, palm):
        """Fingertips in world: R(euler XYZ)·tip + palm_pos (optimize_pregrasp.py:657-669)."""
        tips = self.chain.forward_kinematics(q.float(), self.ee_links, self.ee_offsets)[0].double().view(-1, 4, 3)
        R = euler_xyz(palm[:, 3:])
        return torch.bmm(R, tips.transpose(1, 2)).transpose(1, 2) + palm[:, :3].unsqueeze(1)

    def compute_loss(self, all_tip, q, target, comp, noise):
        """Seven cost terms per pregrasp row (optimize_pregrasp.py:713-739)."""
        g = self.gpis
        dist, std = g.pred(all_tip)
        tar_dist, _ = g.pred(target)
        normal = g.compute_normal(all_tip)
        reward, margin, fnorm, flip = force_eq_reward(
            all_tip, target, comp, self.mu, normal.view(target.shape), noise,
            mass=self.mass, gravity=10.0 if self.gravity else None, COM=self.com)
        c = -reward * 200.0
        center_cost = -contact_margin(all_tip, target, normal, self.mu) * 200.0
        force_cost = -(fnorm * torch.nn.functional.softmin(fnorm, dim=1)).clamp(max=10.0).sum(dim=1)
        ref_cost = (q - self.ref_q).norm(dim=1) * 10.0
        var_cost = self.uncertainty * torch.log(100 * std).max(dim=1)[0]
        dist_cost = 1000 * torch.abs(dist).sum(dim=1)
        tar_cost = 20 * tar_dist.sum(dim=1)
        l = c + dist_cost + tar_cost + center_cost + force_cost + ref_cost + var_cost
        return l, margin, flip

    def closure(self, q, comp, target, palm_pos, palm_ori, noise):
        """One cost+grad eval for all E candidates (optimize_pregrasp.py:741-769).
        ``noise`` [K·E, 3, 3] is the Kabsch ``rand_like`` draw.  Returns
        (loss, total_loss [E], total_margin [E,4], pregrasp_tip [E,4,3], flip [K·E])
        and leaves gradients in the leaves' ``.grad``."""
        E = q.shape[0]
        K = len(self.coeffs)
        palm = torch.hstack([palm_pos, palm_ori])
        pre = self.forward_kinematics(q, palm)
        target_ext = target.repeat(K, 1, 1)
        pre_ext = pre.repeat(K, 1, 1)
        co = self.coeffs.repeat_interleave(E, dim=0)
        all_tip = target_ext + co.view(-1, 4, 1) * (pre_ext - target_ext)
        l, margin, flip = self.compute_loss(all_tip, q.repeat(K, 1), target_ext, comp.repeat(K, 1), noise)
        total_loss = (self.weights.unsqueeze(1) * l.view(-1, E)).sum(dim=0)
        total_margin = (self.weights.view(-1, 1, 1) * margin.view(-1, E, 4)).sum(dim=0)
        pre_dist, _ = self.gpis.pred(pre)
        total_loss = total_loss - pre_dist.sum(dim=1) * 5.0
        if self.optimize_palm:
            palm_dist, _ = self.gpis.pred(palm_pos)
            total_loss = total_loss + 1 / palm_dist
        loss = total_loss.sum()
        loss.backward()
        return loss.detach(), total_loss.detach(), total_margin.detach(), pre.detach(), flip


def collision_loss(chain, anchor_links, anchor_offsets, pairs, q, palm, threshold=0.02, optimize_palm=True):
    """compute_collision_loss (optimize_pregrasp.py:671-701): anchor FK (f32) in world, 1/d for
    anchor pairs closer than ``threshold``, 0.1/z for anchors below z = 0.02, 1/z for a palm
    below z = 0.02 (when the palm is optimised).  Masked terms are multiplied by 0 (so a NaN
    or inf there stays NaN, as in the reference's ``*= 0.0``)."""
    L = len(anchor_links)
    a = chain.forward_kinematics(q.float(), anchor_links, anchor_offsets)[0].double().view(-1, L, 3)
    R = euler_xyz(palm[:, 3:])
    a = torch.bmm(R, a.transpose(1, 2)).transpose(1, 2) + palm[:, :3].unsqueeze(1)
    pr = torch.as_tensor(pairs).long()
    dist = torch.norm(a[:, pr[:, 0]] - a[:, pr[:, 1]], dim=2)
    inv = 1.0 / dist
    inv = torch.where(dist < threshold, inv, inv * 0.0)
    cost = inv.sum(dim=1)
    z = a[:, :, 2]
    zc = 1 / z * 0.1
    cost = cost + torch.where(z < 0.02, zc, zc * 0.0).sum(dim=1)
    if optimize_palm:
        pz = 1 / palm[:, 2]
        cost = cost + torch.where(palm[:, 2] < 0.02, pz, pz * 0.0)
    return cost


def closure_with_grads(problem, q, comp, target, palm, noise):
    """Convenience: runs the oracle closure on fresh leaves, returns a dict of numpy arrays."""
    q = torch.as_tensor(q, dtype=F64).clone().requires_grad_(True)
    comp = torch.as_tensor(comp, dtype=F64).clone().requires_grad_(True)
    target = torch.as_tensor(target, dtype=F64).clone().requires_grad_(True)
    palm = torch.as_tensor(palm, dtype=F64)
    pp = palm[:, :3].clone().requires_grad_(True)
    po = palm[:, 3:].clone().requires_grad_(True)
    noise = torch.as_tensor(noise, dtype=F64)
    loss, tl, tm, pre, flip = problem.closure(q, comp, target, pp, po, noise)
    return dict(loss=float(loss), total_loss=tl.numpy(), total_margin=tm.numpy(), pregrasp_tip=pre.numpy(),
                flip=flip.numpy(), grad_q=q.grad.numpy(), grad_comp=comp.grad.numpy(),
                grad_target=target.grad.numpy(), grad_palm_pos=pp.grad.numpy(), grad_palm_ori=po.grad.numpy())


# ----------------------------------------------------------------------------- Kin mode (config 4)
def kin_sdf_loop(chain, ee_links, ee_offsets, palm_offset, ref_q, q0, target0, comp0, mu, faces, faces_deflate, sdf,
                 noise_tape, iters, mass=0.1, com=(0.0, 0.0, 0.0), gravity=True, adam_state=None, state_out=None):
    """KinGraspOptimizer.optimize with optimize_target=True (optimize_pregrasp.py:152-227), in the
    reference's float32: FK (:143-150, fresh-state — the loop only calls it recursively), the three
    TorchSDF calls per iteration (:186-188) through ``sdf(points, faces) -> (sqdist, sign, normals,
    clst)`` (autograd w.r.t. points; the caller passes the C oracle of the TorchSDF kernel), blended
    signed normals (:190-191), force_eq_reward with the replayed Kabsch noise (:192-198), the six cost
    terms (:199-208), backward, best-iterate tracking (:214-222) and Adam (:171-173, :223).
    ``tar_sign`` is read as [E, T] (the reference's [E·T] broadcast at :207 runs only for E = 1, where
    the two agree).  ``adam_state`` (optional): (step, m_q, v_q, m_target, v_target, m_comp, v_comp) — resume from
    another implementation's loop state after ``step`` iterations (Adam's moments and step count, as torch.optim.Adam
    keeps them), so the loop continues from exactly that state (``noise_tape`` then holds the draws from that
    iteration on).  ``state_out`` (optional dict): receives the loop state after the last step in the same form
    (``adam_state`` plus the parameters q, target, comp).  Returns (loss [iters, E], opt_q, opt_comp, opt_target,
    success flag)."""
    q = torch.as_tensor(q0, dtype=F32).clone().requires_grad_(True)
    comp = torch.as_tensor(comp0, dtype=F32).clone().requires_grad_(True)
    target = torch.as_tensor(target0, dtype=F32).clone().requires_grad_(True)
    palm = torch.as_tensor(palm_offset, dtype=F32).view(1, 3)
    ref = torch.tensor(list(map(float, ref_q)))
    optim = torch.optim.Adam([{"params": q, "lr": 2e-3}, {"params": target, "lr": 1e-5},
                              {"params": comp, "lr": 0.2}])
    if adam_state is not None:
        step, *mv = adam_state
        for prm, m, v in zip((q, target, comp), mv[0::2], mv[1::2]):
            optim.state[prm] = {"step": torch.tensor(float(step)), "exp_avg": torch.as_tensor(m, dtype=F32).clone(),
                                "exp_avg_sq": torch.as_tensor(v, dtype=F32).clone()}
    E, T = target.shape[0], target.shape[1]
    opt_q, opt_comp, opt_target = q.detach().clone(), comp.detach().clone(), target.detach().clone()
    opt_value = torch.full((E,), float("inf"))
    opt_margin = None
    trace = []
    for s in range(iters):
        optim.zero_grad()
        tips = (chain.forward_kinematics(q, ee_links, ee_offsets)[0].view(-1, 3) + palm).view(-1, 3)
        _, sign1, n1, _ = sdf(tips, faces_deflate)
        dist, sign2, n2, _ = sdf(tips, faces)
        tar_dist, tar_sign, _, _ = sdf(target.reshape(-1, 3), faces)
        normal = 0.5 * sign1.unsqueeze(1) * n1 + 0.5 * sign2.unsqueeze(1) * n2
        normal = normal / normal.norm(dim=1).unsqueeze(1)
        noise = torch.as_tensor(noise_tape[s]).to(F32)
        reward, margin, fnorm, _ = force_eq_reward(tips.view(E, T, 3), target, comp, mu, normal.view(E, T, 3).detach(),
                                                   noise, mass=mass, gravity=10.0 if gravity else None, COM=com)
        c = -reward * 5.0
        center_cost = (tips.view(E, T, 3).mean(dim=1) - target.mean(dim=1)).norm(dim=1) * 10.0
        force_cost = -(fnorm * torch.nn.functional.softmin(fnorm, dim=1)).clamp(max=1.0).sum(dim=1)
        ref_cost = (q - ref).norm(dim=1) * 10.0
        dist_cost = 1000 * torch.sqrt(dist).view(E, T).sum(dim=1)
        tar_dist_cost = 10 * (tar_sign.view(E, T) * torch.sqrt(tar_dist).view(E, T)).sum(dim=1)
        l = c + dist_cost + tar_dist_cost + center_cost + force_cost + ref_cost
        l.sum().backward()
        trace.append(l.detach().clone())
        with torch.no_grad():
            flag = l < opt_value
            if flag.any():
                opt_margin = margin.detach().clone()
                opt_value[flag] = l[flag]
                opt_q[flag] = q[flag]
                opt_target[flag] = target[flag]
                opt_comp[flag] = comp[flag]
        optim.step()
    if state_out is not None:
        st = [optim.state[prm] for prm in (q, target, comp)]
        state_out["adam_state"] = (int(st[0]["step"]), *[t.clone() for x in st for t in (x["exp_avg"], x["exp_avg_sq"])])
        state_out.update(q=q.detach().clone(), target=target.detach().clone(), comp=comp.detach().clone())
    return torch.stack(trace), opt_q, opt_comp, opt_target, bool((opt_margin > 0.0).all())


# ----------------------------------------------------------------------------- SDF mode
def sdf_mode_loop(tips0, target0, comp0, mu, faces, faces_deflate, sdf, noise_tape, iters, box_lb, box_ub,
                  mass=0.1, com=(0.0, 0.0, 0.0), gravity=True):
    """SDFGraspOptimizer.optimize with optimize_target=True (optimize_pregrasp.py:240-320), in the reference's
    float32: the three TorchSDF calls per iteration (:273-275) through ``sdf(points, faces)`` (the C oracle of
    the kernel), blended signed normals (:277-278), force_eq_reward with the replayed Kabsch noise (:279-287),
    the five cost terms (:288-296), backward, best-iterate tracking (:301-309), RMSprop (:250-253, :310) and the
    bounding-box clamps of tips and targets (:312-314).  ``tar_sign`` is read as [E, T] (the reference's [E·T]
    broadcast at :296 runs only for E = 1).  Returns (loss [iters, E], opt_tips, opt_comp, opt_target, flag)."""
    tips = torch.as_tensor(tips0, dtype=F32).clone().requires_grad_(True)
    comp = torch.as_tensor(comp0, dtype=F32).clone().requires_grad_(True)
    target = torch.as_tensor(target0, dtype=F32).clone().requires_grad_(True)
    lb = torch.as_tensor(box_lb, dtype=F32).view(-1, 3)
    ub = torch.as_tensor(box_ub, dtype=F32).view(-1, 3)
    optim = torch.optim.RMSprop([{"params": tips, "lr": 1e-3}, {"params": target, "lr": 1e-3},
                                 {"params": comp, "lr": 0.2}])
    E, T = tips.shape[0], tips.shape[1]
    opt_tips, opt_comp, opt_target = tips.detach().clone(), comp.detach().clone(), target.detach().clone()
    opt_value = torch.full((E,), float("inf"))
    opt_margin = None
    trace = []
    for s in range(iters):
        optim.zero_grad()
        all_tip = tips.view(-1, 3)
        _, sign1, n1, _ = sdf(all_tip, faces_deflate)
        dist, sign2, n2, _ = sdf(all_tip, faces)
        tar_dist, tar_sign, _, _ = sdf(target.reshape(-1, 3), faces)
        normal = 0.5 * sign1.unsqueeze(1) * n1 + 0.5 * sign2.unsqueeze(1) * n2
        normal = normal / normal.norm(dim=1).unsqueeze(1)
        noise = torch.as_tensor(noise_tape[s]).to(F32)
        reward, margin, fnorm, _ = force_eq_reward(tips, target, comp, mu, normal.view(E, T, 3).detach(), noise,
                                                   mass=mass, gravity=10.0 if gravity else None, COM=com)
        c = -reward * 5.0
        center_cost = (tips.mean(dim=1) - target.mean(dim=1)).norm(dim=1) * 10.0
        force_cost = -(fnorm * torch.nn.functional.softmin(fnorm, dim=1)).clamp(max=1.0).sum(dim=1)
        dist_cost = 1000 * torch.sqrt(dist).view(E, T).sum(dim=1)
        tar_dist_cost = 10 * (torch.sqrt(tar_dist).view(E, T) * tar_sign.view(E, T)).sum(dim=1)
        l = c + dist_cost + tar_dist_cost + center_cost + force_cost
        l.sum().backward()
        trace.append(l.detach().clone())
        with torch.no_grad():
            flag = l < opt_value
            if flag.any():
                opt_margin = margin.detach().clone()
                opt_value[flag] = l[flag]
                opt_tips[flag] = tips[flag]
                opt_target[flag] = target[flag]
                opt_comp[flag] = comp[flag]
        optim.step()
        with torch.no_grad():
            tips.clamp_(min=lb, max=ub)
            target.clamp_(min=lb, max=ub)
    return torch.stack(trace), opt_tips, opt_comp, opt_target, bool((opt_margin > 0.0).all())
