"""Builds the ``cdx_problem`` descriptor for the prob-mode closure (include/cdx.h).

Every constant is rounded the way the reference materialises it:
``cos_mu`` via ``torch.sqrt(1/(1+torch.tensor(mu)**2))`` (float32, optimize_pregrasp.py:111),
pregrasp coefficients float32 (:644), weights float64 (:645), ``ref_q`` float32 (:634),
the dummy gravity spring's COM / target / stiffness as float32 tensors (:88-94).
"""
from __future__ import annotations

import ctypes

import torch

from ._native import MAX_DOFS, MAX_LEVELS, MAX_TIPS, CdxGpis, CdxProblem

DEFAULT_COEFFS = [[0.8, 0.8, 0.8, 0.8]] * 3
DEFAULT_WEIGHTS = [0.1, 0.8, 0.1]


def cos_friction(mu):
    return float(torch.sqrt(1 / (1 + torch.tensor(mu) ** 2)))


def build_problem(chain_desc, gpis_desc=None, ref_q=(), coeffs=DEFAULT_COEFFS, weights=DEFAULT_WEIGHTS, mu=1,
                  mass=0.1, com=(0.0, 0.0, 0.0), gravity=True, M=2.0, gravity_acc=10.0, uncertainty=20.0,
                  optimize_palm=True):
    """chain_desc: a ``cdx_chain`` with the fingertips (and offsets) set; gpis_desc: ``cdx_gpis``."""
    p = CdxProblem()
    ctypes.memmove(ctypes.byref(p.chain), ctypes.byref(chain_desc), ctypes.sizeof(chain_desc))
    if gpis_desc is not None:
        ctypes.memmove(ctypes.byref(p.gpis), ctypes.byref(gpis_desc), ctypes.sizeof(CdxGpis))
    T = chain_desc.n_tips
    coeffs_t = torch.tensor(coeffs)  # float32 like the reference
    K = coeffs_t.shape[0]
    if not 1 <= K <= MAX_LEVELS or coeffs_t.shape[1] != T or T > MAX_TIPS:
        raise ValueError(f"pregrasp coefficients must be [K<= {MAX_LEVELS}, {T}]")
    if len(weights) != K:
        raise ValueError("one pregrasp weight per level")
    rows = []
    p.n_levels = K
    for k in range(K):
        row = tuple(coeffs_t[k].tolist())
        if row not in rows:
            rows.append(row)
        p.level_query[k] = rows.index(row)
        for f in range(T):
            p.coeff[k][f] = float(coeffs_t[k, f])
    p.n_query_levels = len(rows)
    w = torch.tensor(weights).double()
    for k in range(K):
        p.weight[k] = float(w[k])
    rq = torch.tensor([float(v) for v in ref_q])  # float32
    if len(rq) != chain_desc.n_dofs or len(rq) > MAX_DOFS:
        raise ValueError(f"ref_q must have {chain_desc.n_dofs} entries")
    for i, v in enumerate(rq.tolist()):
        p.ref_q[i] = v
    p.cos_mu = cos_friction(mu)
    p.gravity = 1 if gravity else 0
    p.optimize_palm = 1 if optimize_palm else 0
    com32 = torch.tensor([float(c) for c in com], dtype=torch.float64).float()
    for i in range(3):
        p.com[i] = float(com32[i])
    p.dummy_target_z = float(torch.tensor(-M, dtype=torch.float32))
    p.dummy_comp = float((gravity_acc * mass / M * torch.ones(1))[0])
    p.uncertainty = float(uncertainty)
    return p


def build_collision(anchor_chain_desc, pairs, threshold=0.02, palm_term=True, floor_z=0.02):
    """``cdx_collision`` for compute_collision_loss (optimize_pregrasp.py:671-701): the anchor links
    as the chain's tips, collision pairs as anchor indices, the 0.02 pair and floor thresholds."""
    from ._native import MAX_PAIRS, CdxCollision
    if len(pairs) > MAX_PAIRS:
        raise ValueError(f"at most {MAX_PAIRS} collision pairs")
    c = CdxCollision()
    ctypes.memmove(ctypes.byref(c.chain), ctypes.byref(anchor_chain_desc), ctypes.sizeof(anchor_chain_desc))
    c.n_pairs = len(pairs)
    for i, (lft, rgt) in enumerate(pairs):
        c.pairs[i][0], c.pairs[i][1] = int(lft), int(rgt)
    c.pair_threshold = float(threshold)
    c.floor_z = float(floor_z)
    c.palm_term = int(bool(palm_term))
    return c
