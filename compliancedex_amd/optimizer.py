"""Drop-in for ``ProbabilisticGraspOptimizer`` (optimize_pregrasp.py:614-839) on MI355X.

``closure`` is ONE native call (cdx_closure: FK → GPIS queries → fused cost + analytic
backward) that writes the five parameter gradients straight into ``.grad``; ``optimize``
keeps the reference's loop (Adam, best-iterate tracking after step 20, compliance and
target clamps).  Module constants mirror optimize_pregrasp.py:13-30.
"""
from __future__ import annotations

import warnings

import numpy as np
import torch

from . import _native as N
from .problem import build_collision, build_problem
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


class _Collision(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, palm, desc):
        lib = N.load()
        E = q.shape[0]
        f64 = dict(dtype=torch.float64, device=q.device)
        qd = q.detach().to(torch.float64).contiguous()
        pd = palm.detach().to(torch.float64)
        pp, po = pd[:, :3].contiguous(), pd[:, 3:].contiguous()
        if qd.shape != (E, desc.chain.n_dofs) or pd.shape != (E, 6):
            raise ValueError("compute_collision_loss: q must be [E, n_dofs] and palm poses [E, 6]")
        cost = torch.empty(E, **f64)
        g_q, g_pp, g_po = torch.empty(E, desc.chain.n_dofs, **f64), torch.empty(E, 3, **f64), torch.empty(E, 3, **f64)
        N.check(lib.cdx_collision_loss(desc, E, N.ptr(qd), N.ptr(pp), N.ptr(po), N.ptr(cost), N.ptr(g_q), N.ptr(g_pp),
                                       N.ptr(g_po), 0, N.stream_ptr(q.device)), "cdx_collision_loss")
        ctx.save_for_backward(g_q, torch.cat([g_pp, g_po], 1))
        ctx.dtypes = (q.dtype, palm.dtype)
        return cost

    @staticmethod
    def backward(ctx, g):
        g_q, g_palm = ctx.saved_tensors
        g = g.to(torch.float64).unsqueeze(1)
        return (g * g_q).to(ctx.dtypes[0]), (g * g_palm).to(ctx.dtypes[1]), None


class ProbabilisticGraspOptimizer:
    def __init__(self, robot_urdf, ee_link_names, ee_link_offsets=EE_OFFSETS, palm_offset=WRIST_OFFSET,
                 num_iters=1000, optimize_target=False, ref_q=None, tip_bounding_box=(FINGERTIP_LB, FINGERTIP_UB),
                 pregrasp_coefficients=((0.8, 0.8, 0.8, 0.8),) * 3, pregrasp_weights=(0.1, 0.8, 0.1),
                 anchor_link_names=None, anchor_link_offsets=None, collision_pairs=None,
                 collision_pair_threshold=0.02, mass=0.1, com=(0.0, 0.0, 0.0), gravity=True, uncertainty=20.0,
                 optimize_palm=False, device="cuda", seed=0, collision=False):
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
        self.collision_pairs = [tuple(map(int, pr)) for pr in collision_pairs] if collision_pairs is not None else None
        if collision_pairs is not None:
            cp = torch.tensor(collision_pairs).long().to(self.device)
            self.collision_pair_left, self.collision_pair_right = cp[:, 0], cp[:, 1]
        self.collision_pair_threshold = collision_pair_threshold
        self.collision = bool(collision)
        self._collision = None
        self.mass, self.com, self.gravity, self.uncertainty = mass, list(com), gravity, uncertainty
        self._chain_desc = self.robot_model._descriptor(self.ee_link_names, self.ee_link_offsets)
        self._problem = self._problem_state = self._problem_key = None
        self._ws = None
        self._last_ws = None  # workspace of the most recent closure (the optimiser's or a graph's own)
        self._seed = int(seed)
        self.screen_repairs = 0  # screened closures of optimise loops that repaired themselves (failed a check)
        self.last_screen_report = None
        self._graphs = {}
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

    def collision_descriptor(self):
        """cdx_collision for the anchor links / pairs given at construction (:626-632)."""
        if self._collision is None:
            if self.anchor_link_names is None or self.collision_pairs is None:
                raise ValueError("compute_collision_loss needs anchor_link_names and collision_pairs")
            self._collision = build_collision(self.robot_model._descriptor(self.anchor_link_names,
                                                                           self.anchor_link_offsets),
                                              self.collision_pairs, self.collision_pair_threshold, self.optimize_palm)
        return self._collision

    def compute_collision_loss(self, joint_angles, palm_poses=None):
        """Pairwise / floor / palm proximity penalty (:671-701; commented out of the reference
        closure at :765, enabled here by ``collision=True``), differentiable w.r.t. the joint
        angles and the palm pose through cdx_collision_loss."""
        if palm_poses is None:
            palm_poses = self.palm_offset
        return _Collision.apply(joint_angles, palm_poses, self.collision_descriptor())

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

    def screen_report(self, gpis, E, friction_mu=1):
        """Verification record of the last closure over E candidates (cdx_closure_screen_report, one
        stream-ordered device→host copy): exact / audited rows, margin misses, audit flips, faults,
        whether the closure repaired itself, the largest estimate error in units of its margin, the
        smallest normalised gap left unaudited, and the same summed since the workspace's last reset —
        or None when the closure ran the full fp64 pass."""
        if self._last_ws is None:
            return None
        rep = N.CdxScreenReport()
        N.check(N.load().cdx_closure_screen_report(self.problem(gpis, friction_mu), E, N.ptr(self._last_ws), rep,
                                                   N.stream_ptr(self._last_ws.device)), "cdx_closure_screen_report")
        return rep.as_dict() if rep.screened else None

    def screen_stats(self, gpis, E, friction_mu=1):
        """The main counts of ``screen_report``: exact_rows, bound_misses, screened_rows (+ audit)."""
        r = self.screen_report(gpis, E, friction_mu)
        if r is None:
            return None
        return {k: r[k] for k in ("exact_rows", "bound_misses", "screened_rows", "audited_rows", "audit_misses",
                                  "audit_flips", "faults", "max_ratio", "max_ratio_audit", "repaired", "min_gap")}

    def _reset_screen(self, p, E, ws):
        N.check(N.load().cdx_closure_screen_reset(p, E, N.ptr(ws), N.stream_ptr(ws.device)), "cdx_closure_screen_reset")

    def _ensure_ws(self, p, E, dev):
        need = N.load().cdx_closure_workspace(p, E)
        if self._ws is None or self._ws.numel() < need:
            self._ws = torch.empty(need, dtype=torch.uint8, device=dev)
            self._reset_screen(p, E, self._ws)

    def _closure_into(self, p, q, comp, target, pp, po, noise, out, seed=None, ws=None):
        """cdx_closure on contiguous f64 device tensors, writing into the preallocated ``out``.
        ``seed``: the Kabsch-noise key (default: the next value of this optimiser's counter).
        ``ws``: a caller-owned workspace (a captured hipGraph's own), else the optimiser's."""
        lib = N.load()
        E = q.shape[0]
        if ws is None:
            self._ensure_ws(p, E, q.device)
            ws = self._ws
        if seed is None:
            self._seed += 1
            seed = self._seed
        self._last_ws = ws
        stream = N.stream_ptr(q.device)
        N.check(lib.cdx_closure(p, E, N.ptr(q), N.ptr(comp), N.ptr(target), N.ptr(pp), N.ptr(po), N.ptr(noise),
                                seed, N.ptr(ws), N.ptr(out["total_loss"]), N.ptr(out["total_margin"]),
                                N.ptr(out.get("pregrasp_tip")), N.ptr(out["g_q"]), N.ptr(out["g_comp"]),
                                N.ptr(out["g_target"]), N.ptr(out["g_palm_pos"]), N.ptr(out["g_palm_ori"]),
                                N.ptr(out.get("flip")), stream), "cdx_closure")
        if self.collision:  # total_loss += compute_collision_loss(q, palm) (:765, enabled)
            N.check(lib.cdx_collision_loss(self.collision_descriptor(), E, N.ptr(q), N.ptr(pp), N.ptr(po),
                                           N.ptr(out["total_loss"]), N.ptr(out["g_q"]), N.ptr(out["g_palm_pos"]),
                                           N.ptr(out["g_palm_ori"]), 1, stream), "cdx_collision_loss")

    @staticmethod
    def _outputs(E, T, D, K, dev, with_pre=True):
        f64 = dict(dtype=torch.float64, device=dev)
        out = dict(total_loss=torch.empty(E, **f64), total_margin=torch.empty(E, T, **f64),
                   g_q=torch.empty(E, D, **f64), g_comp=torch.empty(E, T, **f64), g_target=torch.empty(E, T, 3, **f64),
                   g_palm_pos=torch.empty(E, 3, **f64), g_palm_ori=torch.empty(E, 3, **f64),
                   flip=torch.empty(K * E, dtype=torch.int32, device=dev))
        if with_pre:
            out["pregrasp_tip"] = torch.empty(E, T, 3, **f64)
        return out

    def closure(self, joint_angles, compliance, target_pose, palm_poses, palm_oris, friction_mu, gpis, num_envs,
                kabsch_noise=None):
        """One cost+grad eval for all candidates (:741-769).  ``kabsch_noise`` [K·E, 3, 3]
        replays the reference's ``rand_like(H)`` draw; by default it is drawn on device."""
        if self.optim is not None:
            self.optim.zero_grad()
        p = self.problem(gpis, friction_mu)
        E = int(num_envs)
        dev = joint_angles.device
        q = joint_angles.detach().to(torch.float64).contiguous()
        comp = compliance.detach().to(torch.float64).contiguous()
        target = target_pose.detach().to(torch.float64).contiguous()
        pp = palm_poses.detach().to(torch.float64).contiguous()
        po = palm_oris.detach().to(torch.float64).contiguous()
        T, D = p.chain.n_tips, p.chain.n_dofs
        if q.shape != (E, D) or comp.shape != (E, T) or target.shape != (E, T, 3) or pp.shape != (E, 3) or po.shape != (E, 3):
            raise ValueError("closure input shapes do not match num_envs / the hand")
        noise = None
        if kabsch_noise is not None:
            noise = kabsch_noise.to(dtype=torch.float64, device=dev).contiguous()
            if noise.numel() != p.n_levels * E * 9:
                raise ValueError("kabsch_noise must be [K*E, 3, 3]")
        out = self._outputs(E, T, D, p.n_levels, dev)
        self._closure_into(p, q, comp, target, pp, po, noise, out)
        grads = (out["g_q"], out["g_comp"], out["g_target"], out["g_palm_pos"], out["g_palm_ori"])
        for param, grad in zip((joint_angles, compliance, target_pose, palm_poses, palm_oris), grads):
            if param.requires_grad and param.is_leaf:
                grad = grad.to(param.dtype)
                param.grad = grad if param.grad is None else param.grad + grad
        self.pregrasp_tip_pose = out["pregrasp_tip"]
        self.total_loss = out["total_loss"]
        self.total_margin = out["total_margin"]
        self.kabsch_flip = out["flip"]  # det(V·Uᵀ) < 0 mask per (level, candidate) (:64)
        return out["total_loss"].sum()

    # -------------------------------------------------------------- optimize
    def optimize(self, init_joint_angles, target_pose, compliance, friction_mu, gpis, verbose=True,
                 noise_tape=None, fused=True, init_palm=None, graph=False, step_hook=None):
        """The reference's optimisation loop (:771-839).  ``fused=True`` (default): per iteration
        one cdx_closure + one cdx_optimizer_step (Adam, best iterate, clamps on device, no host
        sync); ``fused=False``: the same loop with torch.optim.Adam.  ``noise_tape``: optional
        per-iteration Kabsch noise tensors (parity replay).  ``init_palm`` [E, 6]: start from these
        palm poses instead of ``palm_offset`` (the annealing outer loop's proposals).  ``graph=True``
        (fused only): capture the whole loop once per (E, problem) as a hipGraph and replay it.
        ``step_hook(s, out, state)`` (fused, eager only): called after closure s with its output
        buffers and the parameter buffers / Kabsch noise it ran on (tests: per-step checks)."""
        if init_palm is not None:
            saved = self.palm_offset
            self.palm_offset = init_palm.detach().to(torch.float64)
            try:
                return self.optimize(init_joint_angles, target_pose, compliance, friction_mu, gpis, verbose,
                                     noise_tape, fused, graph=graph, step_hook=step_hook)
            finally:
                self.palm_offset = saved
        if fused:
            return self._optimize_fused(init_joint_angles, target_pose, compliance, friction_mu, gpis, verbose,
                                        noise_tape, graph, step_hook)
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
        p = self.problem(gpis, friction_mu)  # the loop's cumulative screen record starts at zero
        self._ensure_ws(p, num_envs, joint_angles.device)
        self._reset_screen(p, num_envs, self._ws)
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
        self.last_screen_report = self.screen_report(gpis, num_envs, friction_mu) if self.num_iters else None
        return opt_joint_angle, opt_compliance, opt_target_pose, opt_palm_poses, opt_margin

    def adam_config(self):
        """Param groups of optimize (:782-792) with torch.optim.Adam defaults."""
        cfg = N.CdxAdam()
        lrs = [1e-3, 0.2, 2e-3 if self.optimize_target else 0.0, 1e-4 if self.optimize_palm else 0.0,
               1e-4 if self.optimize_palm else 0.0]
        for i, v in enumerate(lrs):
            cfg.lr[i] = v
        cfg.beta1, cfg.beta2, cfg.eps = 0.9, 0.999, 1e-8
        cfg.comp_min = 80.0
        lb = self.tip_bounding_box[0].reshape(-1).double().tolist()
        ub = self.tip_bounding_box[1].reshape(-1).double().tolist()
        for j in range(len(lb)):
            cfg.target_lb[j], cfg.target_ub[j] = lb[j], ub[j]
        cfg.clamp_target = 1
        cfg.best_after = 20
        return cfg

    def _optimize_fused(self, init_joint_angles, target_pose, compliance, friction_mu, gpis, verbose, noise_tape,
                        graph=False, step_hook=None):
        """Device-resident loop: per iteration one cdx_closure + one cdx_optimizer_step, with the
        Kabsch-noise key and Adam's step count in device loop counters (cdx_loop), so the loop is
        the same whether launched eagerly or replayed from a captured hipGraph (``graph=True``;
        captured once per (E, problem), replayed on later calls).

        Screened closures verify and, when a check fails, repair themselves on the device (cdx_closure:
        every all-tip row through the exact pass, the unscreened selection), so every step is the full
        fp64 path's; the loop's cumulative record is read once at the end (one host sync) into
        ``last_screen_report``, and ``screen_repairs`` counts the repaired closures."""
        res = self._optimize_fused_once(init_joint_angles, target_pose, compliance, friction_mu, gpis, verbose,
                                        noise_tape, graph, step_hook)
        rep = self.screen_report(gpis, init_joint_angles.shape[0], friction_mu)
        self.last_screen_report = rep
        if rep is not None and rep["cum_repairs"]:
            self.screen_repairs += rep["cum_repairs"]
            warnings.warn(f"{rep['cum_repairs']} of {rep['cum_closures']} screened closures failed a check and "
                          f"repaired themselves (exact pass over every row)")
        return res

    def _optimize_fused_once(self, init_joint_angles, target_pose, compliance, friction_mu, gpis, verbose,
                             noise_tape, graph=False, step_hook=None):
        lib = N.load()
        p = self.problem(gpis, friction_mu)
        E = init_joint_angles.shape[0]
        T, D, K = p.chain.n_tips, p.chain.n_dofs, p.n_levels
        dev = init_joint_angles.device
        f64 = dict(dtype=torch.float64, device=dev)
        if graph and noise_tape is not None:
            raise ValueError("graph=True draws the Kabsch noise on device; noise_tape needs graph=False")
        if graph and step_hook is not None:
            raise ValueError("step_hook needs graph=False (a replayed graph has no host steps)")
        # A captured graph replays raw device pointers: each cache entry owns its workspace and
        # holds the GPIS state it captured (so neither is freed or reused while the entry lives;
        # the id() in the key cannot be recycled while the entry references the object).
        key = (E, id(self._problem_state), float(friction_mu), self.num_iters)
        cache = self._graphs.get(key) if graph else None
        if cache is None:
            z = torch.zeros
            cache = dict(q=z(E, D, **f64), comp=z(E, T, **f64), target=z(E, T, 3, **f64), pp=z(E, 3, **f64),
                         po=z(E, 3, **f64), loop=torch.zeros(2, dtype=torch.int64, device=dev))
            cache["out"] = self._outputs(E, T, D, K, dev, with_pre=False)
            for k in ("m_q", "v_q"):
                cache[k] = z(E, D, **f64)
            for k in ("m_comp", "v_comp", "opt_margin"):
                cache[k] = z(E, T, **f64)
            for k in ("m_target", "v_target"):
                cache[k] = z(E, T, 3, **f64)
            for k in ("m_palm_pos", "v_palm_pos", "m_palm_ori", "v_palm_ori"):
                cache[k] = z(E, 3, **f64)
            cache.update(opt_value=z(E, **f64), opt_q=z(E, D, **f64), opt_comp=z(E, T, **f64),
                         opt_target=z(E, T, 3, **f64), opt_palm=z(E, 6, **f64))
            if graph:
                cache["ws"] = torch.empty(lib.cdx_closure_workspace(p, E), dtype=torch.uint8, device=dev)
                cache["state"], cache["problem"] = self._problem_state, p
        c, out = cache, cache["out"]
        # (re)initialise the loop state in place — the captured graph reads these buffers
        c["q"].copy_(init_joint_angles.detach())
        c["comp"].copy_(compliance.detach())
        c["target"].copy_(target_pose.detach())
        c["pp"].copy_(self.palm_offset[:, :3])
        c["po"].copy_(self.palm_offset[:, 3:])
        for k in ("m_q", "v_q", "m_comp", "v_comp", "m_target", "v_target", "m_palm_pos", "v_palm_pos", "m_palm_ori",
                  "v_palm_ori", "opt_margin"):
            c[k].zero_()
        c["opt_value"].fill_(float("inf"))
        c["opt_q"].copy_(init_joint_angles.detach())
        c["opt_comp"].copy_(c["comp"])
        c["opt_target"].copy_(c["target"])
        c["opt_palm"].copy_(self.palm_offset)
        c["loop"][0] = self._seed  # fresh noise keys per call, identical eager / replayed
        c["loop"].view(torch.int32)[2] = -1
        self._seed += self.num_iters
        # the loop's cumulative screen record starts at zero (outside any captured graph)
        if graph:
            self._reset_screen(p, E, c["ws"])
        else:
            self._ensure_ws(p, E, dev)
            self._reset_screen(p, E, self._ws)
        st = {k: c[k] for k in ("m_q", "v_q", "m_comp", "v_comp", "m_target", "v_target", "m_palm_pos", "v_palm_pos",
                                "m_palm_ori", "v_palm_ori", "opt_value", "opt_margin", "opt_q", "opt_comp",
                                "opt_target", "opt_palm")}
        bufs = N.CdxOptBuffers(q=c["q"].data_ptr(), comp=c["comp"].data_ptr(), target=c["target"].data_ptr(),
                               palm_pos=c["pp"].data_ptr(), palm_ori=c["po"].data_ptr(), g_q=out["g_q"].data_ptr(),
                               g_comp=out["g_comp"].data_ptr(), g_target=out["g_target"].data_ptr(),
                               g_palm_pos=out["g_palm_pos"].data_ptr(), g_palm_ori=out["g_palm_ori"].data_ptr(),
                               total_loss=out["total_loss"].data_ptr(), total_margin=out["total_margin"].data_ptr(),
                               loop=c["loop"].data_ptr(), **{k: v.data_ptr() for k, v in st.items()})
        cfg = self.adam_config()

        def run_loop():
            stream = N.stream_ptr(dev)
            p.loop = c["loop"].data_ptr()
            try:
                for s in range(self.num_iters):
                    noise = None
                    if noise_tape is not None:
                        noise = noise_tape[s].to(**f64).contiguous()
                    self._closure_into(p, c["q"], c["comp"], c["target"], c["pp"], c["po"], noise, out, seed=0,
                                       ws=c.get("ws"))
                    if step_hook is not None:
                        step_hook(s, out, dict(q=c["q"], comp=c["comp"], target=c["target"], pp=c["pp"],
                                               po=c["po"], noise=noise))
                    N.check(lib.cdx_optimizer_step(cfg, bufs, E, D, T, s, stream), "cdx_optimizer_step")
            finally:
                p.loop = None

        if not graph:
            run_loop()
        elif "graph" in cache:
            self._last_ws = c["ws"]
            cache["graph"].replay()
        else:
            # workspace and library state exist before capture; the first call captures AND runs
            side = torch.cuda.Stream(device=dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            g = torch.cuda.CUDAGraph()
            with torch.cuda.stream(side):
                with torch.cuda.graph(g, stream=side):
                    run_loop()
            torch.cuda.current_stream(dev).wait_stream(side)
            cache["graph"] = g
            if len(self._graphs) >= 8:  # bound the graphs (and the states/workspaces they pin)
                self._graphs.pop(next(iter(self._graphs)))
            self._graphs[key] = cache
            g.replay()
        if not self.optimize_target and torch.is_tensor(target_pose):
            target_pose.copy_(c["target"])  # the reference clamps the caller's target in place (:834)
        self.total_loss, self.total_margin = out["total_loss"], out["total_margin"]
        self.best_loss = st["opt_value"].clone()
        if verbose:
            print("Margin:", st["opt_margin"])
        return (st["opt_q"].clone(), st["opt_comp"].clone(), st["opt_target"].clone(), st["opt_palm"].clone(),
                st["opt_margin"].clone())
