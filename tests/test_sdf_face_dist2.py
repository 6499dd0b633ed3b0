"""The culled TorchSDF kernels evaluate a face through its precomputed record (cdx_sdf.h face_dist2: the
edge vectors, squared lengths and edge normals of point_face computed once per face).  The contract is
bit-identity with point_face, the restatement of the reference's per-face body
(unbatched_triangle_distance_cuda.cu:201-237) the oracle and the brute-force paths use.  Checked here on
the host build (same header, FP contraction off) over random pairs and over points placed on and around
the region boundaries — the edge parameters at 0 and 1 and a few ulps either side, vertices, edge
midpoints, tiny and large faces.  CPU only.  (A division-free classification of the edge parameters
passed this check but ran the GPU kernel 12 % slower — profiles/r04x_config4_divfree_ab.jsonl.)"""
import ctypes as C

import numpy as np

from tests._host import host, p


def _check(pts, faces):
    pts = np.ascontiguousarray(pts, np.float32)
    faces = np.ascontiguousarray(faces, np.float32)
    n = len(pts)
    d_rec, d_ref = np.zeros(n, np.float32), np.zeros(n, np.float32)
    host().cdxh_face_dist2(p(pts), p(faces), C.c_int64(n), p(d_rec), p(d_ref))
    bad = d_rec.view(np.uint32) != d_ref.view(np.uint32)
    assert not bad.any(), (int(bad.sum()), pts[bad][:3], faces[bad][:3], d_rec[bad][:3], d_ref[bad][:3])


def _faces(rng, n, scale):
    v = rng.standard_normal((n, 3, 3)) * scale
    e1, e2 = v[:, 1] - v[:, 0], v[:, 2] - v[:, 0]
    keep = np.linalg.norm(np.cross(e1, e2), axis=1) > 1e-3 * scale * scale  # the culled path's faces
    return v[keep]


def test_face_dist2_random_pairs_bitwise():
    rng = np.random.default_rng(1)
    for scale in (1e-3, 0.05, 1.0, 300.0):
        f = _faces(rng, 200_000, scale)
        centre = f.mean(1)
        pts = centre + rng.standard_normal((len(f), 3)) * scale * rng.choice([0.01, 0.3, 1.0, 5.0], (len(f), 1))
        _check(pts, f)


def test_face_dist2_region_boundaries_bitwise():
    """Points whose edge parameter lands on or next to 0 and 1 (in float, as the kernel computes it), off
    the edge by various distances in- and out-of-plane, plus vertices and edge midpoints."""
    rng = np.random.default_rng(2)
    f = _faces(rng, 60_000, 0.05).astype(np.float32)
    out = []
    for (a, b) in ((0, 1), (1, 2), (2, 0)):
        va, vb = f[:, a], f[:, b]
        e = vb - va
        nrm = np.cross(f[:, 1] - f[:, 0], f[:, 2] - f[:, 1])
        nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
        side = np.cross(nrm, e)
        side /= np.linalg.norm(side, axis=1, keepdims=True)
        for t in (0.0, 1.0):
            for k in (-4, -2, -1, 0, 1, 2, 4):
                tt = np.float32(t) + np.float32(k) * np.float32(2.0 ** -24)
                for off in (0.0, 1e-7, 1e-4, 1e-2):
                    for sgn in (-1.0, 1.0):
                        q = va + tt * e + sgn * off * side + off * nrm * rng.choice([-1, 1], (len(f), 1))
                        out.append((q, f))
        out.append((va, f))
        out.append((0.5 * (va + vb), f))
    pts = np.concatenate([o[0] for o in out]).astype(np.float32)
    faces = np.concatenate([o[1] for o in out])
    _check(pts, faces)
