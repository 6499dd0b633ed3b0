"""TorchSDF: the C oracle and the host build of the kernel's per-face code agree bit for bit,
including degenerate faces (NaN) and exact ties.  CPU only."""
import os

import numpy as np

from tests import _host, _sdf_oracle
from tests._helpers import DATA


def _points(rng, faces, n):
    lo, hi = faces.reshape(-1, 3).min(0), faces.reshape(-1, 3).max(0)
    span = hi - lo
    return (lo - 0.2 * span + 1.4 * span * rng.random((n, 3))).astype(np.float32)


def _same(a, b):
    return np.array_equal(a.view(np.uint32) if a.dtype == np.float32 else a,
                          b.view(np.uint32) if b.dtype == np.float32 else b)


def test_sdf_host_matches_oracle_bitwise():
    rng = np.random.default_rng(0)
    for mesh in ("cube", "sphere42", "banana"):
        faces = np.load(os.path.join(DATA, "meshes", f"{mesh}_faces.npy"))
        if mesh == "banana":
            faces = faces[:1500]
        pts = _points(rng, faces, 300)
        pts[:10] = faces[:10, 0]          # exactly on vertices
        pts[10:20] = faces[:10].mean(1)   # on faces
        o = _sdf_oracle.forward(pts, faces)
        h = _host.sdf_forward(pts, faces)
        for a, b in zip(o, h):
            assert _same(a, b)


def test_sdf_degenerate_faces_tile_rule():
    rng = np.random.default_rng(1)
    faces = rng.random((1100, 3, 3)).astype(np.float32)
    faces[0] = faces[0, 0]          # zero-area face at the start of tile 0 → NaN distance
    faces[512, 1] = faces[512, 0]   # degenerate edge at the start of tile 1
    faces[700] = faces[3]           # duplicate face → exact tie, first index must win
    pts = rng.random((200, 3)).astype(np.float32)
    o = _sdf_oracle.forward(pts, faces)
    h = _host.sdf_forward(pts, faces)
    for a, b in zip(o, h):
        assert np.array_equal(a.view(np.uint8), b.view(np.uint8))


def test_sdf_normal_invariant_cpu():
    """tests/normal.py:36-39 of TorchSDF: normals·2·sqrt(d) equals the distance gradient."""
    rng = np.random.default_rng(2)
    faces = np.load(os.path.join(DATA, "meshes", "sphere42_faces.npy"))
    pts = (rng.random((2000, 3)) * 2 - 1).astype(np.float32)
    d, s, n, c, f = _sdf_oracle.forward(pts, faces)
    grad = _sdf_oracle.backward(np.ones_like(d), pts, c)
    direct = n * 2 * np.sqrt(d)[:, None]
    assert np.abs(direct - grad).max() < 5e-7


def test_sdf_double_oracle_invariants_cpu():
    """The C oracle's double instantiation (unbatched_triangle_distance_cuda.cu:282 with scalar_t =
    double): squared distances are float values (the kernel's `float dist`, .cu:237), the TorchSDF
    normal.py invariant holds, and on float32-representable inputs its distance agrees with the float
    instantiation's to float rounding, with the same sign wherever both pick the same face (points
    nearest a shared vertex or edge tie between faces, and the two precisions break ties apart)."""
    rng = np.random.default_rng(3)
    faces = np.load(os.path.join(DATA, "meshes", "sphere42_faces.npy"))
    pts = (rng.random((2000, 3)) * 2 - 1).astype(np.float32)
    d, s, n, c, f = _sdf_oracle.forward_f64(pts.astype(np.float64), faces.astype(np.float64))
    assert d.dtype == np.float64 and np.array_equal(d, d.astype(np.float32).astype(np.float64))
    grad = _sdf_oracle.backward_f64(np.ones_like(d), pts.astype(np.float64), c)
    assert np.abs(n * 2 * np.sqrt(d)[:, None] - grad).max() < 5e-7
    d32, s32, _, _, f32 = _sdf_oracle.forward(pts, faces)
    same = f == f32
    assert same.mean() > 0.9 and np.array_equal(s[same], s32[same])
    assert np.abs(d - d32).max() <= 1e-6 * max(1.0, np.abs(d32).max())
