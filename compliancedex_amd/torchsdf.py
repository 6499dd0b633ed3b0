"""Drop-in for ``torchsdf`` (thirdparty/TorchSDF/torchsdf/sdf.py) on MI355X.

``compute_sdf(points, face_vertices) -> (sqdist, sign, normals, clst_points)``: squared
distance (autograd w.r.t. points), int32 sign, unit (p − c) normal and closest point
(sdf.py:34-64), computed by cdx_sdf_query on a cached prepared mesh / cdx_sdf_backward (float32, the
culled path) or
cdx_sdf_forward_f64 / cdx_sdf_backward_f64 (float64, the reference's double instantiation,
unbatched_triangle_distance_cuda.cu:282).  ``compute_sdf_with_faces`` additionally returns the
argmin face index.
"""
from __future__ import annotations

import torch

from . import _native as N


def index_vertices_by_faces(vertices_features, faces):
    """[V, K] vertex features, [F, 3] faces → [F, 3, K] (sdf.py:5-31)."""
    assert vertices_features.ndim == 2, "vertices_features must have 2 dimensions"
    assert faces.ndim == 2, "faces must have 2 dimensions of shape (num_faces, num_vertices)"
    return vertices_features[faces]


def _check(points, faces):
    if not (points.is_cuda and faces.is_cuda):
        raise RuntimeError("points must be a CUDA tensor")  # unbatched_triangle_distance.cpp:48-53
    if points.dtype not in (torch.float32, torch.float64) or faces.dtype != points.dtype:
        raise RuntimeError("compute_sdf takes float32 or float64 points with face_vertices of the same dtype "
                           "(the reference's dispatch, unbatched_triangle_distance_cuda.cu:32-41, :282)")
    if points.ndim != 2 or points.shape[1] != 3:
        raise RuntimeError(f"points must have shape [P, 3], got {tuple(points.shape)}")
    if faces.ndim != 3 or faces.shape[1:] != (3, 3):
        raise RuntimeError(f"face_vertices must have shape [F, 3, 3], got {tuple(faces.shape)}")


class _MeshCache:
    """Prepared float32 meshes (cdx_sdf_mesh_prepare) of the face tensors queried last: the optimisers
    query the same two meshes every iteration, so the face records / chunk spheres are built once.
    Keyed by the face tensor's storage, shape, device and version counter (an in-place change bumps
    it); an entry holds its face tensor, so the storage cannot be reused while cached."""

    def __init__(self, size=8):
        self.size, self.entries = size, {}

    def get(self, faces):
        key = (faces.data_ptr(), tuple(faces.shape), faces.device.index, faces._version)
        hit = self.entries.pop(key, None)
        if hit is None:
            lib = N.load()
            buf = torch.empty(lib.cdx_sdf_mesh_bytes(faces.shape[0]), dtype=torch.uint8, device=faces.device)
            N.check(lib.cdx_sdf_mesh_prepare(N.ptr(faces), faces.shape[0], N.ptr(buf), N.stream_ptr(faces.device)),
                    "cdx_sdf_mesh_prepare")
            hit = (faces, buf)
            if len(self.entries) >= self.size:
                self.entries.pop(next(iter(self.entries)))
        self.entries[key] = hit  # most recent last
        return hit[1]


_meshes = _MeshCache()


def _forward(points, faces, want_face):
    _check(points, faces)
    lib = N.load()
    points = points.contiguous()
    faces = faces.contiguous()
    P = points.shape[0]
    dist = torch.zeros(P, dtype=points.dtype, device=points.device)
    sign = torch.zeros(P, dtype=torch.int32, device=points.device)
    normals = torch.zeros(P, 3, dtype=points.dtype, device=points.device)
    clst = torch.zeros(P, 3, dtype=points.dtype, device=points.device)
    face = torch.zeros(P, dtype=torch.int32, device=points.device) if want_face else None
    if points.dtype == torch.float32 and P > 0 and faces.shape[0] > 0:
        N.check(lib.cdx_sdf_query(N.ptr(_meshes.get(faces)), N.ptr(faces), faces.shape[0], N.ptr(points), P, N.ptr(dist),
                                  N.ptr(sign), N.ptr(normals), N.ptr(clst), N.ptr(face), N.stream_ptr(points.device)),
                "cdx_sdf_query")
        return dist, sign, normals, clst, face
    fwd = lib.cdx_sdf_forward if points.dtype == torch.float32 else lib.cdx_sdf_forward_f64
    N.check(fwd(N.ptr(points), P, N.ptr(faces), faces.shape[0], N.ptr(dist), N.ptr(sign), N.ptr(normals), N.ptr(clst),
                N.ptr(face), N.stream_ptr(points.device)), "cdx_sdf_forward")
    return dist, sign, normals, clst, face


class _UnbatchedTriangleDistance(torch.autograd.Function):
    @staticmethod
    def forward(ctx, points, face_vertices):
        dist, sign, normals, clst, _ = _forward(points.detach(), face_vertices.detach(), False)
        ctx.save_for_backward(points.detach().contiguous(), clst)
        ctx.mark_non_differentiable(sign, normals, clst)
        return dist, sign, normals, clst

    @staticmethod
    def backward(ctx, grad_dist, grad_sign, grad_normals, grad_clst):
        points, clst = ctx.saved_tensors
        lib = N.load()
        grad_dist = grad_dist.to(points.dtype).contiguous()
        grad_points = torch.zeros_like(points)
        bwd = lib.cdx_sdf_backward if points.dtype == torch.float32 else lib.cdx_sdf_backward_f64
        N.check(bwd(N.ptr(grad_dist), N.ptr(points), N.ptr(clst), points.shape[0], N.ptr(grad_points),
                    N.stream_ptr(points.device)), "cdx_sdf_backward")
        return grad_points, None


def compute_sdf(pointclouds, face_vertices):
    return _UnbatchedTriangleDistance.apply(pointclouds, face_vertices)


def compute_sdf_with_faces(points, face_vertices):
    """Forward only; also returns the argmin face (first minimum, reference tile rule)."""
    with torch.no_grad():
        return _forward(points, face_vertices, True)
