"""CPU study: how many (point, face) pairs does each per-face lower bound leave to evaluate exactly on
config 4's TorchSDF calls (16 384-face banana), if every lane knew its final best from the start?

For a sample of each call's points, every face's exact squared distance is computed (numpy, float64) and
the faces whose lower bound is <= the point's true minimum distance are counted per bound:
  exact   faces within 1e-4 relative of the minimum (the irreducible ties)
  sphere  |p - c_f| - r_f                (the culled kernel's per-face test, margins left out)
  aabb    distance to the face's axis-aligned box
  plane   |n_f . (p - v1_f)|             (distance to the face's plane)
  sph+pl  max(sphere, plane)
  slab    max(plane, in-plane distance to the face's circumscribed disk)
Workloads: 'around' = the config-4 test's fingertips (arm base placed so the tips at q = 0 surround the
banana, q = 0.05 randn) and targets (centre + 0.01 randn); 'far' = round 4's timed Kin loop (arm base at the
origin, q = 0.3 randn)."""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def tri_dist2(p, a, b, c):
    """Squared distance from points p [P, 3] to triangles (a, b, c) [F, 3] -> [P, F] (Ericson 5.1.5)."""
    P = p[:, None, :]
    ab, ac = (b - a)[None], (c - a)[None]
    ap = P - a[None]
    d1, d2 = (ab * ap).sum(-1), (ac * ap).sum(-1)
    bp = P - b[None]
    d3, d4 = (ab * bp).sum(-1), (ac * bp).sum(-1)
    cp = P - c[None]
    d5, d6 = (ab * cp).sum(-1), (ac * cp).sum(-1)
    va = d3 * d6 - d5 * d4
    vb = d5 * d2 - d1 * d6
    vc = d1 * d4 - d3 * d2
    denom = np.where(va + vb + vc == 0, 1e-300, va + vb + vc)
    v = vb / denom
    w = vc / denom
    q = a[None] + ab * v[..., None] + ac * w[..., None]  # interior
    # regions (overwrite in reverse priority)
    with np.errstate(divide="ignore", invalid="ignore"):
        # edge bc
        m = (va <= 0) & (d4 - d3 >= 0) & (d5 - d6 >= 0)
        t = (d4 - d3) / ((d4 - d3) + (d5 - d6))
        q = np.where(m[..., None], b[None] + (c - b)[None] * t[..., None], q)
        m = (vb <= 0) & (d2 >= 0) & (d6 <= 0)
        t = d2 / (d2 - d6)
        q = np.where(m[..., None], a[None] + ac * t[..., None], q)
        m = (vc <= 0) & (d1 >= 0) & (d3 <= 0)
        t = d1 / (d1 - d3)
        q = np.where(m[..., None], a[None] + ab * t[..., None], q)
    q = np.where(((d6 >= 0) & (d5 <= d6))[..., None], np.broadcast_to(c[None], q.shape), q)
    q = np.where(((d3 >= 0) & (d4 <= d3))[..., None], np.broadcast_to(b[None], q.shape), q)
    q = np.where(((d1 <= 0) & (d2 <= 0))[..., None], np.broadcast_to(a[None], q.shape), q)
    return ((P - q) ** 2).sum(-1)


def workload(kind, E, rng):
    from compliancedex_amd.urdf import load_robot
    from tests._helpers import oracle_chain
    D = 23
    links = load_robot("iiwa7_allegro")["config"]["ee_link_name"]
    offs = [[0.0, -0.04, 0.015]] * 3 + [[0.0, -0.05, -0.015]]
    chain, _ = oracle_chain("iiwa7_allegro")
    center = np.load(os.path.join(REPO, "compliancedex_amd", "data", "banana_center.npy"))
    with torch.no_grad():
        tips0 = chain.forward_kinematics(torch.zeros(1, D), links, offs)[0].view(4, 3).double().mean(0).numpy()
        if kind == "around":
            q = torch.from_numpy(0.05 * rng.standard_normal((E, D))).float()
            base = center - tips0
        else:
            q = torch.from_numpy(0.3 * rng.standard_normal((E, D))).float()
            base = np.zeros(3)
        tips = chain.forward_kinematics(q, links, offs)[0].view(-1, 3).double().numpy() + base
    target = (np.tile(center, (E, 4, 1)) + 0.01 * rng.standard_normal((E, 4, 3))).reshape(-1, 3)
    return tips, target


def main():
    from compliancedex_amd.optimizers import TriangleMesh, _face_vertices
    rng = np.random.default_rng(0)
    mesh = TriangleMesh.from_npz(os.path.join(REPO, "compliancedex_amd", "data", "meshes", "banana_mesh.npz"))
    faces = _face_vertices(mesh, "cpu").double().numpy()
    deflated = _face_vertices(TriangleMesh(mesh.vertices, mesh.triangles).scale(0.9, [0, 0, 0]), "cpu").double().numpy()
    n_sample = int(os.environ.get("SAMPLE", "384"))
    for kind in ("around", "far"):
        tips, target = workload(kind, 4096, rng)
        for name, pts, fv in (("tips_vs_deflated", tips, deflated), ("tips_vs_mesh", tips, faces),
                              ("targets_vs_mesh", target, faces)):
            a, b, c = fv[:, 0], fv[:, 1], fv[:, 2]
            cen = 0.5 * (np.minimum(np.minimum(a, b), c) + np.maximum(np.maximum(a, b), c))
            rad = np.sqrt(np.max(np.stack([((v - cen) ** 2).sum(-1) for v in (a, b, c)]), 0))
            nrm = np.cross(b - a, c - a)
            nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
            lo, hi = np.minimum(np.minimum(a, b), c), np.maximum(np.maximum(a, b), c)
            sel = rng.choice(len(pts), n_sample, replace=False)
            counts = {k: [] for k in ("exact", "sphere", "aabb", "plane", "sph+pl", "slab")}
            dmin = []
            for i0 in range(0, n_sample, 32):
                p = pts[sel[i0:i0 + 32]]
                d2 = tri_dist2(p, a, b, c)
                best = d2.min(1)
                dmin.append(np.sqrt(best))
                sb = np.sqrt(best)[:, None]
                cd = np.linalg.norm(p[:, None] - cen[None], axis=-1)
                sph = cd - rad[None]
                box = np.linalg.norm(np.maximum(np.maximum(lo[None] - p[:, None], p[:, None] - hi[None]), 0), axis=-1)
                pl = np.abs(((p[:, None] - a[None]) * nrm[None]).sum(-1))
                inpl = np.sqrt(np.maximum(cd ** 2 - ((p[:, None] - cen[None]) * nrm[None]).sum(-1) ** 2, 0)) - rad[None]
                slab = np.sqrt(pl ** 2 + np.maximum(inpl, 0) ** 2)
                counts["exact"].append((d2 <= best[:, None] * (1 + 1e-4)).sum(1))
                for k, lb in (("sphere", sph), ("aabb", box), ("plane", pl), ("sph+pl", np.maximum(sph, pl)),
                              ("slab", slab)):
                    counts[k].append((lb <= sb).sum(1))
            dmin = np.concatenate(dmin)
            row = {"workload": kind, "call": name, "points_sampled": n_sample, "faces": len(fv),
                   "dist_median_m": float(np.median(dmin)), "dist_p90_m": float(np.quantile(dmin, 0.9))}
            for k, v in counts.items():
                v = np.concatenate(v)
                row[f"{k}_mean"] = float(v.mean())
                row[f"{k}_p90"] = float(np.quantile(v, 0.9))
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
