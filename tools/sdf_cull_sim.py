"""CPU simulation of the culled TorchSDF kernel's work per 64-point wave on config 4's calls, for
alternative bound / visiting strategies (tools/sdf_bound_study.py gives the per-face bound tightness
with a perfect best; this one models the order in which a wave's lanes learn their best).

Per wave of 64 Morton-sorted points (mesh frame, 10 bits per axis), faces in Morton order of their
centroids in 32-face chunks with bounding spheres.  Counted per wave: chunk visits (a chunk some lane
cannot rule out with the chunk sphere bound against its current best), per-face bound tests (32 per
visit: the wave tests every face of a visited chunk), and (lane, face) pairs evaluated (per-lane needs,
compacted).  Strategies:
  cur     upper bound from the chunk spheres, one seed chunk (nearest to the middle lane), chunks in
          Morton order, per-face sphere test              (round 4's sdf_culled2_kernel, one slice)
  slab    cur with the per-face slab bound (plane distance with the in-plane disk offset)
  lane    each lane's own nearest chunk (smallest centre distance) evaluated first for that lane, then
          chunks in Morton order with the slab test
  order   lane, with the wave visiting chunks in increasing order of the wave's smallest lower bound
"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))
from sdf_bound_study import tri_dist2, workload  # noqa: E402

CH = 32
STRATS = os.environ.get("STRATS", "cur,order,cyl,tree").split(",")


def spread10(v):
    v = v.astype(np.uint64) & 1023
    v = (v | (v << 16)) & 0x030000FF
    v = (v | (v << 8)) & 0x0300F00F
    v = (v | (v << 4)) & 0x030C30C3
    v = (v | (v << 2)) & 0x09249249
    return v


def morton(x, lo, hi):
    t = np.clip((x - lo) / (hi - lo), 0, 1)
    k = (t * 1023).astype(np.uint64)
    return spread10(k[:, 0]) | (spread10(k[:, 1]) << 1) | (spread10(k[:, 2]) << 2)


def kd_order(cen, leaf=32):
    """Face order of a median-split k-d tree on the centroids (split the longest extent; left part a
    multiple of `leaf` faces), so every run of `leaf` (or leaf·2^k) consecutive faces is one subtree."""
    out = []

    def rec(idx):
        n = len(idx)
        if n <= leaf:
            out.extend(idx.tolist())
            return
        pts = cen[idx]
        ax = int(np.argmax(pts.max(0) - pts.min(0)))
        half = ((n + 1) // 2 + leaf - 1) // leaf * leaf
        half = min(half, n - 1)
        o = np.argsort(pts[:, ax], kind="stable")
        rec(idx[o[:half]])
        rec(idx[o[half:]])
    rec(np.arange(len(cen)))
    return np.array(out)


class Mesh:
    def __init__(self, fv):
        lo, hi = fv.reshape(-1, 3).min(0), fv.reshape(-1, 3).max(0)
        self.lo, self.hi = lo, hi
        order = kd_order(fv.mean(1)) if os.environ.get("KD") else np.argsort(morton(fv.mean(1), lo, hi), kind="stable")
        fv = fv[order]
        self.fv = fv
        a, b, c = fv[:, 0], fv[:, 1], fv[:, 2]
        self.a, self.b, self.c = a, b, c
        self.cen = 0.5 * (np.minimum(np.minimum(a, b), c) + np.maximum(np.maximum(a, b), c))
        self.rad = np.sqrt(np.max(np.stack([((v - self.cen) ** 2).sum(-1) for v in (a, b, c)]), 0))
        n = np.cross(b - a, c - a)
        self.n = n / np.linalg.norm(n, axis=1, keepdims=True)
        F = len(fv)
        self.C = (F + CH - 1) // CH
        self.ccen = np.zeros((self.C, 3))
        self.crad = np.zeros(self.C)
        for k in range(self.C):
            v = fv[k * CH:(k + 1) * CH].reshape(-1, 3)
            m = 0.5 * (v.min(0) + v.max(0))
            self.ccen[k] = m
            self.crad[k] = np.sqrt(((v - m) ** 2).sum(-1).max())
        # chunk cylinders: axis = area-weighted mean normal of the chunk's faces, through the box centre
        self.cax = np.zeros((self.C, 3))
        self.cmid = np.zeros(self.C)
        self.cth = np.zeros(self.C)
        self.cr = np.zeros(self.C)
        for k in range(self.C):
            sl = slice(k * CH, (k + 1) * CH)
            nn = np.cross(self.b[sl] - self.a[sl], self.c[sl] - self.a[sl]).sum(0)
            ax = nn / max(np.linalg.norm(nn), 1e-30)
            v = fv[sl].reshape(-1, 3) - self.ccen[k]
            h = v @ ax
            self.cax[k] = ax
            self.cmid[k] = 0.5 * (h.min() + h.max())
            self.cth[k] = 0.5 * (h.max() - h.min())
            self.cr[k] = np.sqrt(np.maximum((v ** 2).sum(-1) - h ** 2, 0).max())

    def build_tree(self, leaf=16, branch=16):
        """Leaves of `leaf` faces, top nodes of `branch` leaves, each with a bounding cylinder + sphere."""
        self.leaf, self.branch = leaf, branch
        F = len(self.fv)
        self.nodes = {}
        for lvl, size in (("leaf", leaf), ("top", leaf * branch)):
            n = (F + size - 1) // size
            cen, rad, ax, mid, th, cr = (np.zeros((n, 3)), np.zeros(n), np.zeros((n, 3)), np.zeros(n), np.zeros(n),
                                          np.zeros(n))
            for k in range(n):
                sl = slice(k * size, (k + 1) * size)
                v = self.fv[sl].reshape(-1, 3)
                m = 0.5 * (v.min(0) + v.max(0))
                cen[k] = m
                rad[k] = np.sqrt(((v - m) ** 2).sum(-1).max())
                nn = np.cross(self.b[sl] - self.a[sl], self.c[sl] - self.a[sl]).sum(0)
                a_ = nn / max(np.linalg.norm(nn), 1e-30)
                h = (v - m) @ a_
                ax[k] = a_
                mid[k] = 0.5 * (h.min() + h.max())
                th[k] = 0.5 * (h.max() - h.min())
                cr[k] = np.sqrt(np.maximum(((v - m) ** 2).sum(-1) - ((v - m) @ a_) ** 2, 0).max())
            self.nodes[lvl] = (cen, rad, ax, mid, th, cr)

    def node_lb(self, lvl, p):
        cen, rad, ax, mid, th, cr = self.nodes[lvl]
        d = p[:, None] - cen[None]
        h = (d * ax[None]).sum(-1)
        rho = np.sqrt(np.maximum((d ** 2).sum(-1) - h ** 2, 0))
        dh = np.maximum(np.abs(h - mid[None]) - th[None], 0)
        dr = np.maximum(rho - cr[None], 0)
        return np.maximum(np.sqrt(dh ** 2 + dr ** 2), np.linalg.norm(d, axis=-1) - rad[None])

    def chunk_lb_cyl(self, p):
        d = p[:, None] - self.ccen[None]
        h = (d * self.cax[None]).sum(-1)
        rho = np.sqrt(np.maximum((d ** 2).sum(-1) - h ** 2, 0))
        dh = np.maximum(np.abs(h - self.cmid[None]) - self.cth[None], 0)
        dr = np.maximum(rho - self.cr[None], 0)
        return np.maximum(np.sqrt(dh ** 2 + dr ** 2), np.linalg.norm(d, axis=-1) - self.crad[None])

    def lb_sphere(self, p):
        return np.linalg.norm(p[:, None] - self.cen[None], axis=-1) - self.rad[None]

    def lb_slab(self, p):
        d = p[:, None] - self.cen[None]
        h = (d * self.n[None]).sum(-1)
        pl = np.abs(((p[:, None] - self.a[None]) * self.n[None]).sum(-1))
        inpl = np.sqrt(np.maximum((d ** 2).sum(-1) - h ** 2, 0)) - self.rad[None]
        return np.sqrt(pl ** 2 + np.maximum(inpl, 0) ** 2)


def simulate_tree(mesh, p, d2):
    dist = np.sqrt(d2)
    nl = len(p)
    L, B = mesh.leaf, mesh.branch
    tlb = mesh.node_lb("top", p)          # [64, T]
    llb = mesh.node_lb("leaf", p)         # [64, C]
    flb = mesh.lb_slab(p)                 # [64, F]
    F = len(mesh.fv)
    # greedy descent per lane: min-LB top node, min-LB leaf in it, min-LB face in it: its distance = best0
    tests = {"top": tlb.shape[1], "leaf": 0, "face": 0}
    t0 = tlb.argmin(1)
    lsel = np.array([t0[i] * B + int(np.argmin(llb[i, t0[i] * B:(t0[i] + 1) * B])) for i in range(nl)])
    fsel = np.array([lsel[i] * L + int(np.argmin(flb[i, lsel[i] * L:(lsel[i] + 1) * L])) for i in range(nl)])
    tests["leaf"] += B
    tests["face"] += L
    if os.environ.get("INIT", "greedy") == "greedy":
        best = dist[np.arange(nl), fsel]
        pairs = nl
    else:  # the upper bound over the top nodes only
        cen, rad = mesh.nodes["top"][0], mesh.nodes["top"][1]
        best = (np.linalg.norm(p[:, None] - cen[None], axis=-1) + rad[None]).min(1)
        pairs = 0
    tv = lv = 0
    torder = np.argsort(tlb.min(0)) if os.environ.get("TOPORDER", "sorted") == "sorted" else range(tlb.shape[1])
    for t in torder:
        if not (tlb[:, t] <= best).any():
            continue
        tv += 1
        tests["leaf"] += B
        for l in range(t * B, min((t + 1) * B, llb.shape[1])):
            if not (llb[:, l] <= best).any():
                continue
            lv += 1
            tests["face"] += L
            sl = slice(l * L, min((l + 1) * L, F))
            need = flb[:, sl] <= best[:, None]
            pairs += int(need.sum())
            best = np.minimum(best, np.where(need, dist[:, sl], np.inf).min(1))
    assert np.allclose(best, dist.min(1))
    return tv, lv, tests["top"], tests["leaf"], tests["face"], pairs


def simulate(mesh, p, strategy):
    d2 = tri_dist2(p, mesh.a, mesh.b, mesh.c)            # [64, F]
    if strategy == "tree":
        return simulate_tree(mesh, p, d2)
    dist = np.sqrt(d2)
    cd = np.linalg.norm(p[:, None] - mesh.ccen[None], axis=-1)  # [64, C]
    clb = cd - mesh.crad[None]
    if strategy in ("cyl", "cylall"):
        clb = mesh.chunk_lb_cyl(p)
    cub = cd + mesh.crad[None]
    flb = mesh.lb_sphere(p) if strategy == "cur" else mesh.lb_slab(p)
    best = cub.min(1)                                     # pass 1: upper bound (distance units)
    visits = tests = pairs = 0
    nl = len(p)
    order = list(range(mesh.C))
    if strategy == "cur" or strategy == "slab":
        seed = int(np.argmin(cd[nl // 2]))
        pairs += nl * min(CH, len(mesh.fv) - seed * CH)   # the seed chunk, all lanes
        best = np.minimum(best, dist[:, seed * CH:(seed + 1) * CH].min(1))
    else:
        own = np.argmin(cd, 1)                            # each lane's nearest chunk
        for k in np.unique(own):
            lanes = own == k
            sl = slice(k * CH, (k + 1) * CH)
            visits += 1
            tests += CH
            need = (flb[:, sl] <= best[:, None]) & lanes[:, None]
            pairs += int(need.sum())
            dd = np.where(need, dist[:, sl], np.inf).min(1)
            best = np.minimum(best, dd)
        if strategy in ("order", "cyl", "cylall"):
            order = list(np.argsort(clb.min(0)))
    for k in order:
        if not (clb[:, k] <= best).any():
            continue
        visits += 1
        tests += CH
        sl = slice(k * CH, (k + 1) * CH)
        need = flb[:, sl] <= best[:, None]
        pairs += int(need.sum())
        dd = np.where(need, dist[:, sl], np.inf).min(1)
        best = np.minimum(best, dd)
    assert np.allclose(best, dist.min(1))
    global LANE_CHUNKS
    LANE_CHUNKS.append(float((clb <= best[:, None]).sum(1).mean()))
    return visits, tests, pairs


LANE_CHUNKS = []


def main():
    from compliancedex_amd.optimizers import TriangleMesh, _face_vertices
    rng = np.random.default_rng(1)
    mesh0 = TriangleMesh.from_npz(os.path.join(REPO, "compliancedex_amd", "data", "meshes", "banana_mesh.npz"))
    faces = _face_vertices(mesh0, "cpu").double().numpy()
    deflated = _face_vertices(TriangleMesh(mesh0.vertices, mesh0.triangles).scale(0.9, [0, 0, 0]), "cpu").double().numpy()
    meshes = {"mesh": Mesh(faces), "deflated": Mesh(deflated)}
    for m in meshes.values():
        m.build_tree(int(os.environ.get("LEAF", "16")), int(os.environ.get("BRANCH", "16")))
    n_waves = int(os.environ.get("WAVES", "24"))
    for kind in ("around", "far"):
        tips, target = workload(kind, 16384, rng)
        for name, pts, mk in (("tips_vs_mesh", tips, "mesh"), ("targets_vs_mesh", target, "mesh")):
            m = meshes[mk]
            frame = (pts.min(0), pts.max(0)) if os.environ.get("OWNFRAME") else (m.lo, m.hi)
            srt = pts[np.argsort(morton(pts, *frame), kind="stable")]
            waves = rng.choice(len(srt) // 64, n_waves, replace=False)
            row = {"workload": kind, "call": name, "waves": n_waves}
            for st in STRATS:
                if st == "tree":
                    tot = np.zeros(6)
                    for w in waves:
                        tot += simulate(m, srt[64 * w:64 * w + 64], st)
                    tot /= n_waves
                    row[st] = {"top_visits": round(tot[0], 1), "leaf_visits": round(tot[1], 1),
                               "tests_per_lane": round(tot[2] + tot[3] + tot[4]), "pairs_per_point": round(tot[5] / 64, 1)}
                    continue
                tot = np.zeros(3)
                LANE_CHUNKS.clear()
                for w in waves:
                    tot += simulate(m, srt[64 * w:64 * w + 64], st)
                v, t, pr = tot / n_waves
                row[st] = {"lane_chunks": round(float(np.mean(LANE_CHUNKS)) if LANE_CHUNKS else 0, 1), "visits_per_wave": round(v, 1), "face_tests_per_wave": round(t), "pairs_per_point": round(pr / 64, 1)}
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
