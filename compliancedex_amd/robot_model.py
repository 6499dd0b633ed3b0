"""Drop-in for ``DifferentiableRobotModel`` FK (thirdparty/differentiable-robot-model/
differentiable_robot_model/robot_model.py) on MI355X: ``compute_forward_kinematics``
(:224-264) with the reference's float32 arithmetic and gradient (cdx_fk_forward /
cdx_fk_backward).  Dynamics (ID/FD/ABA/Jacobians, :266-806) are not on the path.
"""
from __future__ import annotations

import torch

from . import _native as N
from .chain import Chain
from .urdf import load_robot


class _FK(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, chain_desc):
        lib = N.load()
        qf = q.detach().to(torch.float32).contiguous()
        B, T = qf.shape[0], chain_desc.n_tips
        pos = torch.empty(B, 3 * T, dtype=torch.float32, device=q.device)
        quat = torch.empty(B, 4 * T, dtype=torch.float32, device=q.device)
        N.check(lib.cdx_fk_forward(chain_desc, N.ptr(qf), B, N.ptr(pos), N.ptr(quat), N.stream_ptr(q.device)),
                "cdx_fk_forward")
        ctx.save_for_backward(qf)
        ctx.chain_desc = chain_desc
        ctx.q_dtype = q.dtype
        ctx.mark_non_differentiable(quat)
        return pos, quat

    @staticmethod
    def backward(ctx, g_pos, g_quat):
        (qf,) = ctx.saved_tensors
        gq = None
        if ctx.needs_input_grad[0] and g_pos is not None:
            lib = N.load()
            gq = torch.empty_like(qf)
            N.check(lib.cdx_fk_backward(ctx.chain_desc, N.ptr(qf), qf.shape[0],
                                        N.ptr(g_pos.to(torch.float32).contiguous()), N.ptr(gq),
                                        N.stream_ptr(qf.device)), "cdx_fk_backward")
            gq = gq.to(ctx.q_dtype)
        return gq, None


class DifferentiableRobotModel(torch.nn.Module):
    """``urdf_path``: a URDF file, or a packaged robot name (allegro, leap, iiwa7_allegro)."""

    def __init__(self, urdf_path: str, name="", device=None):
        super().__init__()
        self.name = name
        self._device = torch.device(device) if device is not None else torch.device("cuda")
        self.chain = Chain(load_robot(urdf_path))
        self._n_dofs = self.chain.n_dofs
        self._name_to_idx_map = dict(self.chain.index)
        self._desc_cache = {}

    def _descriptor(self, link_names, offsets):
        key = (tuple(link_names), None if offsets is None else tuple(tuple(float(v) for v in o) for o in offsets))
        d = self._desc_cache.get(key)
        if d is None:
            d = self._desc_cache[key] = self.chain.descriptor(list(link_names), offsets)
        return d

    def get_joint_limits(self):
        return [dict(lower=b["lower"], upper=b["upper"]) for i, b in enumerate(self.chain.bodies) if self.chain.dof[i] >= 0]

    def compute_forward_kinematics(self, q: torch.Tensor, link_names: list, recursive: bool = False, offsets=None):
        """→ (pos [B, 3L], quat [B, 4L] xyzw), float32 (robot_model.py:224-264).

        ``recursive=True`` returns the same fresh-state result: the reference's recursive
        branch composes with each body's pose left over from the previous call
        (rigid_body.py:111-118) and is used only by the out-of-scope Kin/WC optimizers."""
        if q.device.type != self._device.type:
            raise AssertionError(f"Input argument of different device as module: {q.device}")
        if q.ndim not in (1, 2):
            raise AssertionError("Input tensors must have ndim of 1 or 2.")
        if q.shape[-1] != self._n_dofs:
            raise AssertionError(f"q must have {self._n_dofs} joints")
        if not q.is_cuda:
            raise RuntimeError("compliancedex_amd FK runs on the GPU only")
        squeeze = q.ndim == 1
        q2 = q.unsqueeze(0) if squeeze else q
        pos, quat = _FK.apply(q2, self._descriptor(link_names, offsets))
        if squeeze:
            return pos[0], quat[0]
        return pos, quat
