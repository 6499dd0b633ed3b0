"""Drop-in for ``torchsdf`` (thirdparty/TorchSDF/torchsdf/sdf.py) on MI355X.

``compute_sdf(points, face_vertices) -> (sqdist, sign, normals, clst_points)``: squared
distance (autograd w.r.t. points), int32 sign, unit (p − c) normal and closest point
(sdf.py:34-64), computed by cdx_sdf_forward (one shot) or cdx_sdf_query on a PreparedMesh /
cdx_sdf_backward (float32, the culled path) or
cdx_sdf_forward_f64 / cdx_sdf_backward_f64 (float64, the reference's double instantiation,
unbatched_triangle_distance_cuda.cu:282).  ``compute_sdf_with_faces`` additionally returns the
argmin face index.
"""
from __future__ import annotations

import ctypes as C
import os

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


class PreparedMesh:
    """A float32 triangle mesh prepared once for repeated queries (cdx_sdf_mesh_prepare: face records in the
    order of a k-d tree on the centroids, their disk slabs, the 32-face chunks' and 512-face top nodes'
    bounding cylinders) — the SDF / Kin optimisers query the same two meshes every iteration.

    The handle owns a private copy of the faces: later writes to the caller's tensor (in place, through
    ``.data``, DLPack, raw device pointers or a graph replay) never reach it, so a query always answers for
    the mesh the handle was built from; build a new handle for a changed mesh.  Its query scratch (the points'
    Morton sort) is kept and regrown when a larger batch comes, so a loop at a fixed point count allocates
    nothing per query.  Preparing copies the faces to the host once (a wait on the current stream)."""

    def __init__(self, face_vertices):
        _check(face_vertices.new_zeros(0, 3), face_vertices)
        if face_vertices.dtype != torch.float32 or face_vertices.shape[0] == 0:
            raise RuntimeError("PreparedMesh takes a non-empty float32 [F, 3, 3] face tensor")
        lib = N.load()
        self.faces = face_vertices.detach().contiguous().clone()
        F = self.faces.shape[0]
        self.buf = torch.empty(lib.cdx_sdf_mesh_bytes(F), dtype=torch.uint8, device=self.faces.device)
        stream = N.stream_ptr(self.faces.device)
        N.check(lib.cdx_sdf_mesh_prepare(N.ptr(self.faces), F, N.ptr(self.buf), stream), "cdx_sdf_mesh_prepare")
        kind = C.c_int32(0)
        N.check(lib.cdx_sdf_mesh_flags(N.ptr(self.buf), C.byref(kind), stream), "cdx_sdf_mesh_flags")
        self.kind = kind.value  # SDF_MESH_CULLED, or SDF_MESH_EXACT for a mesh with a NaN-capable face
        self._ws = QueryWorkspace()

    @property
    def num_faces(self):
        return self.faces.shape[0]

    def query(self, points, want_face=False, workspace=None, reuse_order=False, out=None):
        """(sqdist, sign, normals, clst, face | None) of float32 points [P, 3] (cdx_sdf_query).  ``workspace``: a
        QueryWorkspace to sort the points in (default: the mesh's own); ``reuse_order``: walk the points in the order
        the workspace's last sort left (of P points — these same points on another mesh, or earlier positions of
        them) instead of sorting them again.  The results are the same for any order; only the culling's speed
        depends on how close the order keeps nearby points."""
        _check(points, self.faces)
        lib = N.load()
        points = points.detach().contiguous()
        P, dev = points.shape[0], points.device
        if out is not None:  # (dist [P] f32, sign [P] i32, normals [P, 3] f32, clst [P, 3] f32), contiguous
            dist, sign, normals, clst = out
            if not (dist.shape == (P,) and sign.shape == (P,) and normals.shape == (P, 3) and clst.shape == (P, 3) and
                    dist.dtype == normals.dtype == clst.dtype == torch.float32 and sign.dtype == torch.int32 and
                    all(t.is_contiguous() and t.device == dev for t in out)):
                raise RuntimeError("query: out must be (dist [P], sign [P] int32, normals [P, 3], clst [P, 3]) float32")
        else:
            dist = torch.empty(P, dtype=torch.float32, device=dev)
            sign = torch.empty(P, dtype=torch.int32, device=dev)
            normals = torch.empty(P, 3, dtype=torch.float32, device=dev)
            clst = torch.empty(P, 3, dtype=torch.float32, device=dev)
        face = torch.empty(P, dtype=torch.int32, device=dev) if want_face else None
        if P == 0:
            return dist, sign, normals, clst, face
        wsp = workspace or self._ws
        # a mesh with NaN-capable faces (SDF_MESH_EXACT) scans every face: it neither reads nor writes a point order
        walks = self.kind != N.SDF_MESH_EXACT
        ws = wsp.get(P, dev, reuse_order and walks)
        flags = self.kind | (N.SDF_REUSE_ORDER if reuse_order else 0)
        if not reuse_order and walks:
            wsp.order_P = None  # (overwritten by this query's sort; valid again once it is enqueued)
        N.check(lib.cdx_sdf_query(N.ptr(self.buf), N.ptr(self.faces), self.faces.shape[0], N.ptr(points), P,
                                  N.ptr(dist), N.ptr(sign), N.ptr(normals), N.ptr(clst), N.ptr(face),
                                  N.ptr(ws), ws.numel(), flags, N.stream_ptr(dev)), "cdx_sdf_query")
        if not reuse_order and walks:
            wsp.order_P = P  # this query sorted its points: later reuse_order queries of P points may walk that order
        return dist, sign, normals, clst, face


class BatchSchedule:
    """Device state a repeated query_batch carries from one launch to the next (cdx_sdf_query_batch's schedule): each
    point group's walk time, and from it the next launch's order, heaviest groups first.  Regrown (zeroed) when a
    batch with more groups comes; the outputs never depend on it."""

    def __init__(self, every=None):
        """``every``: launches per recomputation of the order (the durations are recorded on every launch; the
        order from a few launches back serves as well, and each recomputation is a launch of its own)."""
        self.buf = None
        self.every = max(1, int(os.environ.get("CDX_SDF_SCHED_EVERY", "4") if every is None else every))
        self.launches = 0

    def keep_order(self):
        """Whether this launch keeps the current order (the count advances)."""
        keep = self.launches % self.every != 0
        self.launches += 1
        return keep

    def get(self, Ps, dev):
        arr = (C.c_int64 * len(Ps))(*Ps)
        need = N.load().cdx_sdf_batch_schedule_bytes(len(Ps), arr)
        if need == 0:
            raise RuntimeError("BatchSchedule: bad point counts")
        if self.buf is None or self.buf.numel() < need or self.buf.device != dev:
            self.buf = torch.zeros(need, dtype=torch.uint8, device=dev)
            self.launches = 0
        groups = sum((P + 63) // 64 for P in Ps)
        if groups != getattr(self, "groups", None):  # (an order for another group count is not used: recompute)
            self.groups, self.launches = groups, 0
        return self.buf


def query_batch(items, schedule=None):
    """Several PreparedMesh queries in one launch (cdx_sdf_query_batch, ≤ 4): ``items`` = [(mesh, points, workspace,
    out)], each workspace already holding its points' order (QueryWorkspace.sort, or a query of the same P points),
    each mesh free of NaN-capable faces (``mesh.kind == SDF_MESH_CULLED``), ``out`` = (dist, sign, normals, clst)
    preallocated as for PreparedMesh.query.  ``schedule``: a BatchSchedule kept across the calls of a loop (the
    heaviest point groups of the last launch start first).  Outputs identical to the separate queries."""
    if not 0 < len(items) <= 4:
        raise RuntimeError("query_batch takes 1 to 4 queries")
    qs = (N.CdxSdfBatchQuery * len(items))()
    keep = []
    dev = None
    for d, (mesh, points, ws, out) in zip(qs, items):
        _check(points, mesh.faces)
        if mesh.kind != N.SDF_MESH_CULLED:
            raise RuntimeError("query_batch: a mesh with NaN-capable faces takes PreparedMesh.query")
        points = points.detach().contiguous()
        P = points.shape[0]
        dev = points.device
        if ws.buf is None or ws.order_P != P:
            raise RuntimeError("query_batch: the workspace holds no order for these points (QueryWorkspace.sort)")
        dist, sign, normals, clst = out
        if not (dist.shape == (P,) and sign.shape == (P,) and normals.shape == (P, 3) and clst.shape == (P, 3) and
                dist.dtype == normals.dtype == clst.dtype == torch.float32 and sign.dtype == torch.int32 and
                all(t.is_contiguous() and t.device == dev for t in out)):
            raise RuntimeError("query_batch: out must be (dist [P], sign [P] int32, normals [P, 3], clst [P, 3]) float32")
        keep.append(points)
        d.mesh, d.faces, d.F = N.ptr(mesh.buf), N.ptr(mesh.faces), mesh.faces.shape[0]
        d.points, d.P = N.ptr(points), P
        d.sqdist, d.sign, d.normals, d.clst, d.face_idx = N.ptr(dist), N.ptr(sign), N.ptr(normals), N.ptr(clst), None
        d.workspace, d.workspace_bytes = N.ptr(ws.buf), ws.buf.numel()
        d.flags = N.SDF_REUSE_ORDER | N.SDF_MESH_CULLED
    sb = schedule.get([d.P for d in qs], dev) if schedule is not None else None
    if sb is not None and schedule.keep_order():
        qs[0].flags |= N.SDF_SCHED_KEEP
    N.check(N.load().cdx_sdf_query_batch(len(items), C.cast(qs, C.c_void_p), N.ptr(sb), 0 if sb is None else sb.numel(),
                                         N.stream_ptr(dev)), "cdx_sdf_query_batch")


class QueryWorkspace:
    """Scratch of cdx_sdf_query (the points' Morton sort), regrown to the largest point count seen; it keeps the
    last sorted order, which a later query of P points may reuse (the same points on another mesh, or the same
    points moved a little — a fused loop's next iterations).  ``order_P`` is the point count of the order it holds
    (None: none) — set only by a sort (``sort``, or a query that sorts: not ``reuse_order``, a mesh without
    NaN-capable faces), cleared when the buffer is regrown; ``reuse_order`` queries and ``query_batch`` require it
    to match, so no walk ever reads an order that was never written."""

    def __init__(self):
        self.buf, self.order_P = None, None

    def sort(self, points):
        """The points' order alone (cdx_sdf_query_order): later queries of these points with ``reuse_order`` — on
        other meshes, on other streams ordered after this call — walk them in it."""
        _check(points, points.new_zeros(1, 3, 3))
        if points.dtype != torch.float32:
            raise RuntimeError("QueryWorkspace.sort takes float32 points")
        points = points.detach().contiguous()
        P, dev = points.shape[0], points.device
        if P == 0:
            return
        buf = self.get(P, dev)
        self.order_P = None
        N.check(N.load().cdx_sdf_query_order(N.ptr(points), P, N.ptr(buf), buf.numel(), N.stream_ptr(dev)),
                "cdx_sdf_query_order")
        self.order_P = P

    def get(self, P, dev, reuse_order=False):
        """The scratch buffer for a query of P points (regrown if needed); ``reuse_order``: the query walks the held
        order, which must be one of P points."""
        if reuse_order and self.order_P != P:
            raise RuntimeError("reuse_order: the workspace holds no order for these points (sort them first)")
        need = N.load().cdx_sdf_query_workspace(P)
        if self.buf is None or self.buf.numel() < need or self.buf.device != torch.device(dev):
            if reuse_order:
                raise RuntimeError("reuse_order: the workspace holds no order for these points")
            self.buf = torch.empty(need, dtype=torch.uint8, device=dev)
            self.order_P = None
        return self.buf


def _forward(points, faces, want_face):
    """One-shot query (cdx_sdf_forward: the mesh's records and bounds are built for this call on the device —
    faces in Morton order of their cubic frame — or the double instantiation's brute-force scan)."""
    if isinstance(faces, PreparedMesh):
        return faces.query(points, want_face)
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
    fwd = lib.cdx_sdf_forward if points.dtype == torch.float32 else lib.cdx_sdf_forward_f64
    N.check(fwd(N.ptr(points), P, N.ptr(faces), faces.shape[0], N.ptr(dist), N.ptr(sign), N.ptr(normals), N.ptr(clst),
                N.ptr(face), N.stream_ptr(points.device)), "cdx_sdf_forward")
    return dist, sign, normals, clst, face


class _UnbatchedTriangleDistance(torch.autograd.Function):
    @staticmethod
    def forward(ctx, points, face_vertices, mesh):
        dist, sign, normals, clst, _ = _forward(points.detach(), mesh if mesh is not None else face_vertices.detach(),
                                                False)
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
        return grad_points, None, None


def compute_sdf(pointclouds, face_vertices):
    """sdf.py:34-64.  ``face_vertices``: a [F, 3, 3] tensor (one-shot query) or a PreparedMesh."""
    if isinstance(face_vertices, PreparedMesh):
        return _UnbatchedTriangleDistance.apply(pointclouds, face_vertices.faces, face_vertices)
    return _UnbatchedTriangleDistance.apply(pointclouds, face_vertices, None)


def compute_sdf_with_faces(points, face_vertices):
    """Forward only; also returns the argmin face (first minimum, reference tile rule).  ``face_vertices``: a
    tensor or a PreparedMesh."""
    with torch.no_grad():
        return _forward(points, face_vertices, True)
