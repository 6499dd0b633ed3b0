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


def synthetic_banana_arrays(n_total=2000):
    pcd = np.load(os.path.join(DATA, "partial_pcd_banana.npy"))
    center = 0.5 * (pcd.min(0) + pcd.max(0))
    n_ext, n_int = 14, 50
    n_surf = n_total - n_ext - n_int
    surf = pcd[np.random.default_rng(0).permutation(len(pcd))[:n_surf]]
    bound = 0.15
    ext = np.array([[-1, -1, -1], [1, -1, -1], [-1, 1, -1], [1, 1, -1], [-1, -1, 1], [1, -1, 1], [-1, 1, 1],
                    [1, 1, 1], [-1, 0, 0], [0, -1, 0], [1, 0, 0], [0, 1, 0], [0, 0, 1], [0, 0, -1]],
                   dtype=np.float64) * bound + center
    w = torch.rand(n_int, n_surf, generator=torch.Generator().manual_seed(0)).double()
    internal = (torch.softmax(w * 30, dim=1) @ torch.from_numpy(surf)).numpy()
    X1 = np.vstack([ext, surf, internal])
    y = np.concatenate([np.full(n_ext, bound), np.zeros(n_surf), np.full(n_int, -bound)])[:, None]
    noise = np.concatenate([np.full(n_ext, 0.2), np.full(n_surf, 0.005), np.full(n_int, 0.1)])
    return X1, y, noise


def synthetic_banana_gpis(n_total=2000, device="cuda"):
    from .gpis import GPIS
    X1, y, noise = synthetic_banana_arrays(n_total)
    g = GPIS(0.08, 1.0)
    g.fit(torch.from_numpy(X1).to(device), torch.from_numpy(y).to(device), noise=torch.from_numpy(noise).to(device))
    g.bias = torch.tensor(1.0, dtype=torch.float64, device=device)
    return g


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


def box_gpis(side=0.065, n_surface=400, device="cuda", seed=0):
    """Config 3's "box": the 0.065 m cube of assets/cube_visualization.urdf:7 (no stored state),
    fitted with the same recipe as the synthetic banana: surface samples (y = 0, noise 0.005),
    14 external points at ±0.15 (y = +0.15, noise 0.2), 50 internal points (y = −0.15, noise 0.1)."""
    from .gpis import GPIS
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
    bound = 0.15
    ext = np.array([[-1, -1, -1], [1, -1, -1], [-1, 1, -1], [1, 1, -1], [-1, -1, 1], [1, -1, 1], [-1, 1, 1],
                    [1, 1, 1], [-1, 0, 0], [0, -1, 0], [1, 0, 0], [0, 1, 0], [0, 0, 1], [0, 0, -1]], float) * bound
    internal = rng.uniform(-0.6 * h, 0.6 * h, (50, 3))
    X1 = np.vstack([ext, surf, internal])
    y = np.concatenate([np.full(14, bound), np.zeros(n_surface), np.full(50, -bound)])[:, None]
    noise = np.concatenate([np.full(14, 0.2), np.full(n_surface, 0.005), np.full(50, 0.1)])
    g = GPIS(0.08, 1.0)
    g.fit(torch.from_numpy(X1).to(device), torch.from_numpy(y).to(device), noise=torch.from_numpy(noise).to(device))
    g.bias = torch.tensor(1.0, dtype=torch.float64, device=device)
    return g


# config 3: one object per GPU; "realsense" (fit on the fly from an absent point cloud) is
# stood in for by the stored dummy state, "box" by box_gpis.
CONFIG3_OBJECTS = ["banana", "mug", "mug2", "hammer", "lego", "coffeebottle", "box", "dummy"]


def config3_gpis(rank, device="cuda"):
    name = CONFIG3_OBJECTS[rank % len(CONFIG3_OBJECTS)]
    return name, (box_gpis(device=device) if name == "box" else stored_gpis(name, device))
