"""Simulated-annealing outer loop over the prob-mode inner optimisation (config 5).

The reference's ``simanneal.py`` is an empty file, so this loop is build-defined (SURVEY §8d
config 5): every outer step perturbs the current joint angles and palm poses with a
temperature-scaled Gaussian, runs ``ProbabilisticGraspOptimizer.optimize`` (the fused
closure + Adam/best-iterate/clamp loop, all on device) from the proposal, and accepts the
optimised proposal per candidate with the Metropolis rule on its best loss
(accept if Δ < 0 or u < exp(−Δ/T); NaN losses are rejected), then cools T ← c·T.  The best
state ever reached is kept per candidate.  No host synchronisation inside the loop.

``anneal_sharded`` runs one shard per rank (one process per GPU) and ends with the same single
all-gather of surviving grasps as ``distributed.optimize_sharded``.
"""
from __future__ import annotations

import torch

from . import distributed as D


class PregraspAnnealer:
    def __init__(self, optimizer, gpis, friction_mu=1, temperature=100.0, cooling=0.8, q_sigma=0.05,
                 palm_pos_sigma=0.005, palm_ori_sigma=0.05, seed=0):
        if getattr(optimizer, "num_iters", 1000) <= 21:
            raise ValueError("the inner optimize() tracks its best iterate only after step 20 (:823): "
                             "num_iters must be > 21")
        self.optimizer, self.gpis, self.friction_mu = optimizer, gpis, friction_mu
        self.temperature, self.cooling = float(temperature), float(cooling)
        self.q_sigma, self.palm_pos_sigma, self.palm_ori_sigma = q_sigma, palm_pos_sigma, palm_ori_sigma
        self.seed = int(seed)

    def run(self, q, target, comp, palm, outer_steps=4):
        """q [E, D], target [E, T, 3], comp [E, T], palm [E, 6] (device tensors) → dict of the best
        state per candidate: q, comp, target, palm, margin, loss (+ ``accepted`` counts)."""
        dev = q.device
        f64 = dict(dtype=torch.float64, device=dev)
        gen = torch.Generator(device=dev).manual_seed(self.seed)
        E = q.shape[0]
        cur = dict(q=q.to(**f64).clone(), target=target.to(**f64).clone(), comp=comp.to(**f64).clone(),
                   palm=palm.to(**f64).clone())
        cur_loss = torch.full((E,), float("inf"), **f64)
        best = {k: v.clone() for k, v in cur.items()}
        best["loss"] = torch.full((E,), float("inf"), **f64)
        best["margin"] = torch.zeros(E, comp.shape[1], **f64)
        accepted = torch.zeros(E, dtype=torch.int64, device=dev)
        T = self.temperature
        for k in range(outer_steps):
            prop = dict(cur)
            if k:
                s = T / self.temperature
                prop["q"] = cur["q"] + s * self.q_sigma * torch.randn(cur["q"].shape, generator=gen, **f64)
                dp = torch.cat([self.palm_pos_sigma * torch.randn(E, 3, generator=gen, **f64),
                                self.palm_ori_sigma * torch.randn(E, 3, generator=gen, **f64)], 1)
                prop["palm"] = cur["palm"] + s * dp
            oq, oc, ot, op, om = self.optimizer.optimize(prop["q"], prop["target"], prop["comp"], self.friction_mu,
                                                         self.gpis, verbose=False, init_palm=prop["palm"])
            loss = self.optimizer.best_loss
            u = torch.rand(E, generator=gen, **f64)
            delta = loss - cur_loss
            acc = torch.isfinite(loss) & ((delta < 0) | (u < torch.exp(-delta / T)))
            accepted += acc.long()
            res = dict(q=oq, target=ot, comp=oc, palm=op)
            for key, v in res.items():
                m = acc.view((-1,) + (1,) * (v.dim() - 1))
                cur[key] = torch.where(m, v.to(torch.float64), cur[key])
            cur_loss = torch.where(acc, loss, cur_loss)
            better = loss < best["loss"]
            for key, v in list(res.items()) + [("margin", om)]:
                m = better.view((-1,) + (1,) * (v.dim() - 1))
                best[key] = torch.where(m, v.to(torch.float64), best[key])
            best["loss"] = torch.where(better, loss, best["loss"])
            T *= self.cooling
        best["accepted"] = accepted
        return best


def anneal_sharded(annealer, q, target, comp, palm, outer_steps=4, object_id=0, capacity=None, group=None):
    """Rank-local annealing of this rank's candidate block, then one all-gather of survivors."""
    import torch.distributed as dist
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    lo, hi = D.shard_range(q.shape[0], rank, world)
    best = annealer.run(q[lo:hi], target[lo:hi], comp[lo:hi], palm[lo:hi], outer_steps)
    buf = D.pack_survivors(capacity or D.default_capacity(q.shape[0], world), object_id, rank, lo, best["loss"], best["margin"], best["q"],
                           best["comp"], best["target"], best["palm"])
    if world == 1:
        return best, D.unpack_records([buf])
    return best, D.all_gather_survivors(buf, group)
