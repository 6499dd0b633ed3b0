"""``compliancedex_amd.torchsdf_c`` — the ``torchsdf._C`` replacement (bindings.cpp:22-27).

GPU: the two in-place entry points driven exactly as the reference's torchsdf/sdf.py:42-64 drives
``_C`` (caller-allocated zero-filled outputs, then ``backward`` on the saved closest points) give
bit-identical results to ``compute_sdf``; CPU: the reference's argument checks (CHECK_CUDA,
CHECK_CONTIGUOUS, the dtype dispatch's AT_ERROR) raise RuntimeError before any launch.
"""
import os

import numpy as np
import pytest
import torch

from tests._helpers import DATA


def _reference_sdf_py(_C, points, face_vertices):
    """torchsdf/sdf.py:40-64 (_UnbatchedTriangleDistanceCuda forward + backward with grad_dist = 1),
    restated with ``_C`` swapped for the shim."""
    num_points = points.shape[0]
    min_dist = torch.zeros((num_points), device=points.device, dtype=points.dtype)
    dist_sign = torch.zeros((num_points), device=points.device, dtype=torch.int32)
    normals = torch.zeros((num_points, 3), device=points.device, dtype=points.dtype)
    clst_points = torch.zeros((num_points, 3), device=points.device, dtype=points.dtype)
    _C.unbatched_triangle_distance_forward_cuda(points, face_vertices, min_dist, dist_sign, normals, clst_points)
    grad_dist = torch.ones_like(min_dist).contiguous()
    grad_points = torch.zeros_like(points)
    _C.unbatched_triangle_distance_backward_cuda(grad_dist, points.contiguous(), clst_points, grad_points)
    return min_dist, dist_sign, normals, clst_points, grad_points


@pytest.mark.gpu
@pytest.mark.parametrize("mesh", ["cube", "banana"])
def test_shim_matches_compute_sdf(mesh):
    import compliancedex_amd.torchsdf_c as _C
    from compliancedex_amd import compute_sdf
    faces = torch.from_numpy(np.load(os.path.join(DATA, "meshes", f"{mesh}_faces.npy"))).cuda()
    rng = np.random.default_rng(3)
    f = faces.cpu().numpy().reshape(-1, 3)
    lo, hi = f.min(0), f.max(0)
    pts = torch.from_numpy((lo - 0.2 * (hi - lo) + 1.4 * (hi - lo) * rng.random((4000, 3))).astype(np.float32)).cuda()
    a = _reference_sdf_py(_C, pts, faces)
    p = pts.clone().requires_grad_(True)
    d, s, n, c = compute_sdf(p, faces)
    d.sum().backward()
    torch.cuda.synchronize()
    for x, y in zip(a, (d.detach(), s, n, c, p.grad)):
        assert torch.equal(x, y)


def test_shim_rejects_like_the_reference():
    import compliancedex_amd.torchsdf_c as _C
    pts = torch.zeros(4, 3)
    faces = torch.zeros(2, 3, 3)
    outs = (torch.zeros(4), torch.zeros(4, dtype=torch.int32), torch.zeros(4, 3), torch.zeros(4, 3))
    with pytest.raises(RuntimeError, match="CUDA"):
        _C.unbatched_triangle_distance_forward_cuda(pts, faces, *outs)
    with pytest.raises(RuntimeError, match="CUDA"):
        _C.unbatched_triangle_distance_backward_cuda(outs[0], pts, outs[2], outs[3])


@pytest.mark.gpu
def test_shim_rejects_double_and_noncontiguous():
    import compliancedex_amd.torchsdf_c as _C
    pts = torch.zeros(4, 3, device="cuda", dtype=torch.float64)
    faces = torch.zeros(2, 3, 3, device="cuda", dtype=torch.float64)
    outs = (torch.zeros(4, device="cuda", dtype=torch.float64), torch.zeros(4, device="cuda", dtype=torch.int32),
            torch.zeros(4, 3, device="cuda", dtype=torch.float64), torch.zeros(4, 3, device="cuda", dtype=torch.float64))
    with pytest.raises(RuntimeError, match="not implemented for 'Float64'"):
        _C.unbatched_triangle_distance_forward_cuda(pts, faces, *outs)
    with pytest.raises(RuntimeError, match="contiguous"):
        _C.unbatched_triangle_distance_forward_cuda(torch.zeros(3, 4, device="cuda").t(), faces.float(),
                                                    *(o.float() if o.dtype == torch.float64 else o for o in outs))


@pytest.mark.gpu
def test_shim_checks_sizes_before_any_launch():
    """CHECK_SIZES (unbatched_triangle_distance.cpp:60-67, :90-94): an undersized or mis-shaped
    output, points that are not [P, 3] or faces that are not [F, 3, 3] raise a RuntimeError and no
    kernel runs — the caller's buffers keep their sentinel (the unchecked version wrote past them)."""
    import compliancedex_amd.torchsdf_c as _C
    dev = "cuda"
    P, F = 64, 8
    pts = torch.rand(P, 3, device=dev)
    faces = torch.rand(F, 3, 3, device=dev)

    def outs():
        return [torch.full((P,), 7.0, device=dev), torch.full((P,), 7, device=dev, dtype=torch.int32),
                torch.full((P, 3), 7.0, device=dev), torch.full((P, 3), 7.0, device=dev)]

    bad_fwd = [
        ("dist", lambda o: o.__setitem__(0, torch.full((P - 1,), 7.0, device=dev))),
        ("dist_sign", lambda o: o.__setitem__(1, torch.full((P // 2,), 7, device=dev, dtype=torch.int32))),
        ("normals", lambda o: o.__setitem__(2, torch.full((P, 2), 7.0, device=dev))),
        ("clst_points", lambda o: o.__setitem__(3, torch.full((P * 3,), 7.0, device=dev))),
    ]
    for arg, mutate in bad_fwd:
        o = outs()
        mutate(o)
        with pytest.raises(RuntimeError, match=f"{arg} must of size"):
            _C.unbatched_triangle_distance_forward_cuda(pts, faces, *o)
        torch.cuda.synchronize()
        assert all(bool((t == 7).all()) for t in o), arg
    with pytest.raises(RuntimeError, match="points must of size"):
        _C.unbatched_triangle_distance_forward_cuda(torch.rand(P, 4, device=dev), faces, *outs())
    with pytest.raises(RuntimeError, match="face_vertices must of size"):
        _C.unbatched_triangle_distance_forward_cuda(pts, torch.rand(F, 9, device=dev), *outs())
    g = torch.ones(P, device=dev)
    for args, arg in (((torch.ones(P - 3, device=dev), pts, outs()[3], outs()[2]), "grad_dist"),
                      ((g, pts, torch.full((P - 1, 3), 7.0, device=dev), outs()[2]), "clst_points"),
                      ((g, pts, outs()[3], torch.full((P, 1), 7.0, device=dev)), "grad_points")):
        with pytest.raises(RuntimeError, match=f"{arg} must of size"):
            _C.unbatched_triangle_distance_backward_cuda(*args)
        torch.cuda.synchronize()
        assert bool((args[3] == 7).all())
    # well-formed calls still run
    o = outs()
    _C.unbatched_triangle_distance_forward_cuda(pts, faces, *o)
    gp = torch.zeros(P, 3, device=dev)
    _C.unbatched_triangle_distance_backward_cuda(g, pts, o[3], gp)
    torch.cuda.synchronize()
    assert bool((o[1].abs() == 1).all()) and torch.isfinite(gp).all()
