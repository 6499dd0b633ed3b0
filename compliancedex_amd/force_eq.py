"""Drop-in for ``force_eq_reward`` (optimize_pregrasp.py:73-118) and the Kabsch fit it calls
(``optimal_transformation_batch``, :49-69) on MI355X: cdx_force_eq_forward / _backward (f64,
one row per lane), differentiable w.r.t. tip poses, target poses and compliances.

Constants are materialised as the reference does: ``cos_mu`` through a float32 tensor (:111);
the dummy gravity spring's tip (COM), target (−M) and stiffness (gravity·mass/M) in float32
tensors (:88-94).  ``current_normal`` is treated as detached (every caller passes GPIS / SDF
normals without a graph).  ``kabsch_noise`` [B, 3, 3] replays the reference's
``rand_like(H)`` draw; by default it is drawn on device (counter-based, keyed per call).
"""
from __future__ import annotations

import itertools

import torch

from . import _native as N
from .problem import cos_friction

_seeds = itertools.count(0x5EED)


def force_eq_descriptor(n_tips, friction_mu, mass=0.4, gravity=None, M=2.0, COM=(0.0, 0.05, 0.0)):
    if COM is None:
        raise NotImplementedError("COM=None (dummy tip at the target mean) is not used by any optimiser")
    p = N.CdxForceEq()
    p.cos_mu = cos_friction(friction_mu)
    p.gravity = 0 if gravity is None else 1
    com32 = torch.tensor([float(c) for c in COM], dtype=torch.float64).float()
    for i in range(3):
        p.com[i] = float(com32[i])
    p.dummy_target_z = float(torch.tensor(-M, dtype=torch.float32))
    p.dummy_comp = float((gravity * mass / M * torch.ones(1))[0]) if gravity is not None else 0.0
    p.n_tips = int(n_tips)
    return p


class _ForceEq(torch.autograd.Function):
    @staticmethod
    def forward(ctx, tip, target, comp, normal, desc, noise, seed):
        lib = N.load()
        B, T = tip.shape[0], tip.shape[1]
        f64 = dict(dtype=torch.float64, device=tip.device)
        args = [t.detach().to(torch.float64).contiguous() for t in (tip, target, comp, normal)]
        nz = None if noise is None else noise.detach().to(torch.float64).contiguous()
        reward = torch.empty(B, **f64)
        margin = torch.empty(B, T, **f64)
        fn = torch.empty(B, T, **f64)
        flip = torch.empty(B, dtype=torch.int32, device=tip.device)
        N.check(lib.cdx_force_eq_forward(desc, B, *(N.ptr(a) for a in args), N.ptr(nz), seed, N.ptr(reward),
                                         N.ptr(margin), N.ptr(fn), N.ptr(flip), N.stream_ptr(tip.device)),
                "cdx_force_eq_forward")
        ctx.save_for_backward(*args, *([nz] if nz is not None else []))
        ctx.has_noise = nz is not None
        ctx.desc, ctx.seed = desc, seed
        ctx.dtypes = (tip.dtype, target.dtype, comp.dtype)
        ctx.mark_non_differentiable(margin, flip)
        return reward, margin, fn, flip

    @staticmethod
    def backward(ctx, g_reward, g_margin, g_fn, g_flip):
        saved = ctx.saved_tensors
        tip, target, comp, normal = saved[:4]
        nz = saved[4] if ctx.has_noise else None
        lib = N.load()
        B = tip.shape[0]
        g_tip, g_target, g_comp = torch.empty_like(tip), torch.empty_like(target), torch.empty_like(comp)
        gr = None if g_reward is None else g_reward.to(torch.float64).contiguous()
        gf = None if g_fn is None else g_fn.to(torch.float64).contiguous()
        N.check(lib.cdx_force_eq_backward(ctx.desc, B, N.ptr(tip), N.ptr(target), N.ptr(comp), N.ptr(normal), N.ptr(nz),
                                          ctx.seed, N.ptr(gr), N.ptr(gf), N.ptr(g_tip), N.ptr(g_target), N.ptr(g_comp),
                                          N.stream_ptr(tip.device)), "cdx_force_eq_backward")
        dt = ctx.dtypes
        return g_tip.to(dt[0]), g_target.to(dt[1]), g_comp.to(dt[2]), None, None, None, None


def force_eq_reward(tip_pose, target_pose, compliance, friction_mu, current_normal, mass=0.4, gravity=None, M=2.0,
                    COM=(0.0, 0.05, 0.0), kabsch_noise=None, return_flip=False):
    """(reward [B], margin [B, T], force_norm [B, T]) — optimize_pregrasp.py:73-118.

    tip_pose, target_pose, current_normal: [B, T, 3]; compliance: [B, T]."""
    for t, what in ((tip_pose, "tip_pose"), (target_pose, "target_pose"), (compliance, "compliance"),
                    (current_normal, "current_normal")):
        if not (torch.is_tensor(t) and t.is_cuda):
            raise RuntimeError(f"{what} must be a CUDA (ROCm) tensor: compliancedex_amd has no CPU path")
    B, T = tip_pose.shape[0], tip_pose.shape[1]
    if tip_pose.shape != (B, T, 3) or target_pose.shape != (B, T, 3) or current_normal.shape != (B, T, 3) or \
            compliance.shape != (B, T):
        raise ValueError("force_eq_reward: tip/target/normal must be [B, T, 3] and compliance [B, T]")
    desc = force_eq_descriptor(T, friction_mu, mass, gravity, M, COM)
    if kabsch_noise is not None and kabsch_noise.numel() != B * 9:
        raise ValueError("kabsch_noise must be [B, 3, 3]")
    reward, margin, fn, flip = _ForceEq.apply(tip_pose, target_pose, compliance, current_normal, desc, kabsch_noise,
                                              next(_seeds))
    if return_flip:
        return reward, margin, fn, flip
    return reward, margin, fn
