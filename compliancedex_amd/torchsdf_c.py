"""``torchsdf._C`` replacement: the reference's native TorchSDF binding on libcdx.so.

The reference's only native FFI on this path is the pybind module ``torchsdf._C``
(thirdparty/TorchSDF/torchsdf/csrc/bindings.cpp:22-27) with two in-place ``void`` entry points that
``torchsdf/sdf.py:42-64`` calls on caller-allocated, zero-filled outputs.  This module keeps their
names, argument order, in-place contract and error behaviour (``CHECK_CUDA`` / ``CHECK_CONTIGUOUS``
/ ``CHECK_SIZES`` → ``RuntimeError`` before any launch, unbatched_triangle_distance.cpp:48-67,
:81-93; the dtype dispatch's ``AT_ERROR`` for anything but its two types,
unbatched_triangle_distance_cuda.cu:32-41), so that

    import compliancedex_amd.torchsdf_c as _C      # in torchsdf/sdf.py, instead of `from torchsdf import _C`

runs the reference's ``sdf.py`` unchanged on gfx950 (cdx_sdf_forward / cdx_sdf_backward).
Both of the reference's dtypes are dispatched: float32 (the live path, optimize_pregrasp.py:165-168)
on the culled kernel, float64 on the double instantiation (cdx_sdf_forward_f64: double arithmetic
except the reference's two ``float``s, .cu:171-173 and :237); anything else gets the dispatch's
``RuntimeError``.
"""
from __future__ import annotations

import torch

from . import _native as N


def _check(name, *tensors):
    for t in tensors:
        if not t.is_cuda:
            raise RuntimeError(f"{name}: all tensors must be CUDA tensors")      # CHECK_CUDA
        if not t.is_contiguous():
            raise RuntimeError(f"{name}: all tensors must be contiguous")        # CHECK_CONTIGUOUS


def _sizes(name, **shapes):
    """CHECK_SIZES (check.h): each tensor's exact shape, in the reference's check order."""
    for arg, (t, want) in shapes.items():
        if tuple(t.shape) != tuple(want):
            raise RuntimeError(f"{name}: {arg} must of size {{{', '.join(map(str, want))}}} "
                               f"(got {list(t.shape)})")


def _dtype(name, points):
    if points.dtype not in (torch.float32, torch.float64):  # AT_ERROR of DISPATCH_INPUT_TYPES (.cu:32-41)
        raise RuntimeError(f"{name} not implemented for '{str(points.dtype).replace('torch.', '').capitalize()}'")


def unbatched_triangle_distance_forward_cuda(points, face_vertices, dist, dist_sign, normals, clst_points):
    """points [P, 3], face_vertices [F, 3, 3] → dist [P] (squared), dist_sign [P] int32, normals [P, 3],
    clst_points [P, 3], written in place (unbatched_triangle_distance.cpp:40-63)."""
    name = "unbatched_triangle_distance_forward_cuda"
    _check(name, points, face_vertices, dist, dist_sign, normals, clst_points)
    if points.dim() < 1 or face_vertices.dim() < 1:
        raise RuntimeError(f"{name}: points and face_vertices must have a leading dimension")
    P, F = points.shape[0], face_vertices.shape[0]
    _sizes(name, points=(points, (P, 3)), face_vertices=(face_vertices, (F, 3, 3)), dist=(dist, (P,)),
           dist_sign=(dist_sign, (P,)), normals=(normals, (P, 3)), clst_points=(clst_points, (P, 3)))
    _dtype(name, points)
    if face_vertices.dtype != points.dtype or dist.dtype != points.dtype or normals.dtype != points.dtype \
            or clst_points.dtype != points.dtype or dist_sign.dtype != torch.int32:
        raise RuntimeError(f"{name}: output dtypes must match the points (dist_sign int32)")
    lib = N.load()
    fwd = lib.cdx_sdf_forward if points.dtype == torch.float32 else lib.cdx_sdf_forward_f64
    N.check(fwd(N.ptr(points), P, N.ptr(face_vertices), face_vertices.shape[0], N.ptr(dist), N.ptr(dist_sign),
                N.ptr(normals), N.ptr(clst_points), None, N.stream_ptr(points.device)), name)


def unbatched_triangle_distance_backward_cuda(grad_dist, points, clst_points, grad_points):
    """grad_points = 2·grad_dist·(points − clst_points), written in place
    (unbatched_triangle_distance.cpp:65-86, unbatched_triangle_distance_cuda.cu:256-270)."""
    name = "unbatched_triangle_distance_backward_cuda"
    _check(name, grad_dist, points, clst_points, grad_points)
    if points.dim() < 1:
        raise RuntimeError(f"{name}: points must have a leading dimension")
    P = points.shape[0]
    _sizes(name, grad_dist=(grad_dist, (P,)), points=(points, (P, 3)), clst_points=(clst_points, (P, 3)),
           grad_points=(grad_points, (P, 3)))
    _dtype(name, points)
    if grad_dist.dtype != points.dtype or clst_points.dtype != points.dtype or grad_points.dtype != points.dtype:
        raise RuntimeError(f"{name}: grad_dist, clst_points and grad_points must match the points' dtype")
    lib = N.load()
    bwd = lib.cdx_sdf_backward if points.dtype == torch.float32 else lib.cdx_sdf_backward_f64
    N.check(bwd(N.ptr(grad_dist), N.ptr(points), N.ptr(clst_points), points.shape[0], N.ptr(grad_points),
                N.stream_ptr(points.device)), name)
