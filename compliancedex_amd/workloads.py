"""Synthetic workloads of BASELINE.json's configs, shared by bench.py,
``__graft_entry__.smoke`` and the tests.

* ``synthetic_banana_gpis``: the N = 2000 banana GPIS fitted by the in-repo recipe of
  optimize_pregrasp.py:904-922 (14 external points at ±0.15, surface points from
  partial_pcd/banana.npy, 50 softmax-weighted internal points; noise 0.2 / 0.005 / 0.1).
* ``prob_inputs``: candidates as ``__main__`` builds them (:885-999, --use_config banana):
  wrist rows WRIST_OFFSET[i mod 6] shifted to the object centre, q = ref_q (+ N(0, 0.1²)
  beyond the first 6), compliance [10, 10, 10, 20], targets at the centre (optionally spread).
"""
from __future__ import annotations

import os

import numpy as np
import torch

DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")


EXTERNAL_DIRS = np.array([[-1, -1, -1], [1, -1, -1], [-1, 1, -1], [1, 1, -1], [-1, -1, 1], [1, -1, 1], [-1, 1, 1],
                          [1, 1, 1], [-1, 0, 0], [0, -1, 0], [1, 0, 0], [0, 1, 0], [0, 0, 1], [0, 0, -1]],
                         dtype=np.float64)


def recipe_arrays(surf, center, n_int=50, bound=0.15, seed=0):
    """The in-repo fit recipe (optimize_pregrasp.py:904-922) on given surface points: 14 external
    points at ±``bound`` around ``center`` (y = +bound, noise 0.2), the surface (y = 0, noise
    0.005), ``n_int`` internal points = softmax(30·U)·surface (y = −bound, noise 0.1)."""
    n_surf = len(surf)
    ext = EXTERNAL_DIRS * bound + center
    w = torch.rand(n_int, n_surf, generator=torch.Generator().manual_seed(seed)).double()
    internal = (torch.softmax(w * 30, dim=1) @ torch.from_numpy(np.ascontiguousarray(surf))).numpy()
    X1 = np.vstack([ext, surf, internal])
    y = np.concatenate([np.full(len(ext), bound), np.zeros(n_surf), np.full(n_int, -bound)])[:, None]
    noise = np.concatenate([np.full(len(ext), 0.2), np.full(n_surf, 0.005), np.full(n_int, 0.1)])
    return X1, y, noise


def synthetic_banana_arrays(n_total=2000):
    pcd = np.load(os.path.join(DATA, "partial_pcd_banana.npy"))
    center = 0.5 * (pcd.min(0) + pcd.max(0))
    surf = pcd[np.random.default_rng(0).permutation(len(pcd))[:n_total - 14 - 50]]
    return recipe_arrays(surf, center)


def fitted_gpis(X1, y, noise, device="cuda"):
    """GPIS(0.08, 1.0) fitted on the device with bias 1 (the recipe's ``gpis.bias``)."""
    from .gpis import GPIS
    g = GPIS(0.08, 1.0)
    g.fit(torch.from_numpy(X1).to(device), torch.from_numpy(y).to(device), noise=torch.from_numpy(noise).to(device))
    g.bias = torch.tensor(1.0, dtype=torch.float64, device=device)
    return g


def synthetic_banana_gpis(n_total=2000, device="cuda"):
    return fitted_gpis(*synthetic_banana_arrays(n_total), device=device)


def stored_gpis(name, device="cuda"):
    from .gpis import GPIS
    g = GPIS(0.08, 1.0)
    g.load_state_data(f"{name}_state", device=device)
    return g


WRIST_OFFSET = np.array([[-0.06, 0.0, 0.05, 0.0, 0.0, 0.0],
                         [-0.04, 0.03, 0.05, 0.0, 0.0, -np.pi / 4],
                         [-0.01, 0.0, 0.05, 0.0, 0.0, np.pi / 4],
                         [0.1, 0.06, 0.03, -np.pi / 2, np.pi / 2, 0.0],
                         [-0.0, -0.06, 0.05, 0.0, 0.0, np.pi / 2],
                         [0.02, -0.04, 0.05, 0.0, 0.0, 3 * np.pi / 4]])


def prob_inputs(ref_q, E, seed=0, spread=True, center=None):
    """numpy (q [E,D], comp [E,4], target [E,4,3], palm [E,6])."""
    if center is None:
        center = np.load(os.path.join(DATA, "banana_center.npy"))
    W = WRIST_OFFSET.copy()
    W[:, 0] += center[0]
    W[:, 1] += center[1]
    W[:, 2] += 2 * center[2]
    W[:, 1] += 0.015          # banana config.json wrist_y
    W[:, 2] += 0.11 - 0.02    # wrist_z - floor_offset
    rng = np.random.default_rng(seed)
    palm = W[np.arange(E) % len(W)]
    ref_q = np.asarray(ref_q, dtype=np.float64)
    q = np.tile(ref_q, (E, 1))
    target = np.tile(center, (E, 4, 1)).astype(np.float64)
    if E > len(W):
        q = q + 0.1 * rng.standard_normal(q.shape)
        palm = palm + np.concatenate([0.005 * rng.standard_normal((E, 3)), 0.05 * rng.standard_normal((E, 3))], 1)
    if spread:
        target = target + 0.01 * rng.standard_normal(target.shape)
    comp = np.tile(np.array([10.0, 10.0, 10.0, 20.0]), (E, 1))
    return q, comp, target, palm


def box_surface(side=0.065, n_surface=400, seed=0):
    """Uniform samples on the faces of the 0.065 m cube of assets/cube_visualization.urdf:7."""
    rng = np.random.default_rng(seed)
    h = side / 2
    face = rng.integers(0, 6, n_surface)
    uv = rng.uniform(-h, h, (n_surface, 2))
    surf = np.zeros((n_surface, 3))
    for i, (f, (u, v)) in enumerate(zip(face, uv)):
        ax, sgn = f // 2, (1 if f % 2 else -1)
        p = [u, v]
        p.insert(ax, sgn * h)
        surf[i] = p
    return surf, rng


def box_arrays(side=0.065, n_surface=400, seed=0):
    """Config 3's "box" (no stored state), reduced size: ``n_surface`` cube-face samples (y = 0,
    noise 0.005), 14 external points at ±0.15 (y = +0.15, noise 0.2), 50 internal points uniform
    in the inner 60 % of the cube (y = −0.15, noise 0.1).  Returns numpy (X1, y, noise)."""
    surf, rng = box_surface(side, n_surface, seed)
    h = side / 2
    bound = 0.15
    ext = EXTERNAL_DIRS * bound
    internal = rng.uniform(-0.6 * h, 0.6 * h, (50, 3))
    X1 = np.vstack([ext, surf, internal])
    y = np.concatenate([np.full(14, bound), np.zeros(n_surface), np.full(50, -bound)])[:, None]
    noise = np.concatenate([np.full(14, 0.2), np.full(n_surface, 0.005), np.full(50, 0.1)])
    return X1, y, noise


def box_gpis(side=0.065, n_surface=400, device="cuda", seed=0):
    """GPIS(0.08, 1.0) fitted on ``box_arrays`` (bias 1, as the synthetic banana)."""
    return fitted_gpis(*box_arrays(side, n_surface, seed), device=device)


# Config 3: one object per GPU.  Two sources per object:
#   "fit" (default, bench and scaling): an N = 2000 GPIS per object with the config-2 recipe —
#     banana = config 2's synthetic state itself (so the 1-GPU run IS config 2); hammer, lego, mug,
#     mug2 from 1 936 points sampled on their meshes, coffeebottle from its observed point cloud
#     (data/config3_surface.npz, tools/import_assets.py); box from its cube; "realsense" (fitted on
#     the fly in the reference from an absent point cloud) from the stored dummy state's surface
#     points, resampled with 1 mm jitter.  Every rank then does config 2's per-GPU work.
#   "stored": the reference's stored states (N = 196…401), the 400-point box, dummy for realsense.
CONFIG3_OBJECTS = ["banana", "mug", "mug2", "hammer", "lego", "coffeebottle", "box", "dummy"]


def config3_arrays(name, n_total=2000):
    """numpy (X1, y, noise) of config 3's N = ``n_total`` GPIS for one object."""
    if name == "banana":
        return synthetic_banana_arrays(n_total)
    n_surf = n_total - 14 - 50
    rng = np.random.default_rng(CONFIG3_OBJECTS.index(name))
    if name == "box":
        surf, _ = box_surface(n_surface=n_surf, seed=1)
    elif name == "dummy":
        d = np.load(os.path.join(DATA, "gpis_states", "dummy_state.npz"))
        y1 = d["y1"].reshape(-1)
        pts = d["X1"][y1 == -1.0]
        surf = pts[rng.integers(0, len(pts), n_surf)] + 1e-3 * rng.standard_normal((n_surf, 3))
    else:
        surf = np.load(os.path.join(DATA, "config3_surface.npz"))[name][:n_surf]
    return recipe_arrays(surf, 0.5 * (surf.min(0) + surf.max(0)))


def config3_gpis(rank, device="cuda", source="fit", n_total=2000):
    """(name, GPIS) of rank ``rank``'s object (see CONFIG3_OBJECTS for the two sources)."""
    name = CONFIG3_OBJECTS[rank % len(CONFIG3_OBJECTS)]
    if source == "fit":
        return name, fitted_gpis(*config3_arrays(name, n_total), device=device)
    return name, (box_gpis(device=device) if name == "box" else stored_gpis(name, device))


def surface_center(gpis):
    """AABB centre of a GPIS's surface points (the most frequent label, y1 = −bias: 0-level set),
    the object centre ``__main__`` derives from the mesh (:885-888)."""
    X1 = gpis.X1.detach().cpu().numpy()
    y1 = gpis.y1.detach().cpu().numpy().reshape(-1)
    vals, counts = np.unique(y1, return_counts=True)
    surf = X1[y1 == vals[np.argmax(counts)]]
    return 0.5 * (surf.min(0) + surf.max(0))


def config3_inputs(gpis, ref_q, E, seed):
    """Config 3's per-object candidates: ``prob_inputs`` around the object's surface centre."""
    return prob_inputs(ref_q, E, seed=seed, spread=True, center=surface_center(gpis))


# Config 4's SDF / Kin leg: the KinGraspOptimizer iteration on iiwa7_allegro (23 DOF, the arm + Allegro chain,
# depth 13) against the 16 384-face banana mesh, E = 16 384 candidates.  The arm base ("palm offset") is
# placed so the fingertips at q = 0 surround the banana; q = 0.05·N(0, 1) per joint; targets at the banana's
# centre + 1 cm noise; compliance [10, 10, 10, 20].  Three TorchSDF calls per iteration (:186-188):
# 4E fingertips vs the deflated and the true mesh, 4E targets vs the true mesh.
CONFIG4_OFFSETS = [[0.0, -0.04, 0.015]] * 3 + [[0.0, -0.05, -0.015]]


def config4_kin_inputs(E=16384, seed=44, device="cuda", q_scale=0.05):
    """(links, offsets, palm_offset [3] f32, q [E, 23], target [E, 4, 3], comp [E, 4]) — float32 numpy."""
    from .robot_model import DifferentiableRobotModel
    from .urdf import load_robot
    D = 23
    links = load_robot("iiwa7_allegro")["config"]["ee_link_name"]
    center = np.load(os.path.join(DATA, "banana_center.npy"))
    tips0 = DifferentiableRobotModel("iiwa7_allegro", device=device).compute_forward_kinematics(
        torch.zeros(1, D, device=device), links, offsets=CONFIG4_OFFSETS)[0].view(4, 3).double().mean(0).cpu().numpy()
    rng = np.random.default_rng(seed)
    q = (q_scale * rng.standard_normal((E, D))).astype(np.float32)
    target = (np.tile(center, (E, 4, 1)) + 0.01 * rng.standard_normal((E, 4, 3))).astype(np.float32)
    comp = np.tile(np.array([10.0, 10.0, 10.0, 20.0], np.float32), (E, 1))
    return links, CONFIG4_OFFSETS, (center - tips0).astype(np.float32), q, target, comp


def banana_mesh():
    from .optimizers import TriangleMesh
    return TriangleMesh.from_npz(os.path.join(DATA, "meshes", "banana_mesh.npz"))
