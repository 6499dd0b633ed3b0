"""Multi-GPU layer: one process per GPU, candidates sharded, no
collective inside the inner loop; one all-gather of fixed-capacity "surviving grasp"
records after ``optimize``.

The closure is a sum of independent per-candidate terms (optimize_pregrasp.py:767), so
each rank optimises its own block of candidates (or its own object, config 3) with the
GPIS state and kinematic chain replicated.  At the end, every rank packs the candidates
whose best-iterate margins are all positive (the reference's success test,
``opt_margin > 0``, :226/:319/:405/:510/:611) into a fixed-capacity float64 record
buffer with a count header — RCCL has no all-gatherv — and one ``all_gather`` (RCCL over
xGMI under the ``nccl`` backend; gloo on CPU in tests) gives every rank the global set.

Record layout (float64, RECORD_FIELDS + D + 5·T entries, ≈ 344 B for Allegro):
  [object_id, rank, candidate_id, best_loss, survive, margin[T], q[D], comp[T], target[T·3], palm[6]]
Row 0 of a rank's buffer is the header: [stored count, true survivor count, capacity, 0, …]; the
two counts differ when more candidates survived than the buffer holds (``overflow``).

Every rank must pass an equal-shaped buffer to ``all_gather`` (RCCL sizes its receive buffers from
the local one), so the default capacity is the same on every rank: ⌈total / world⌉.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

RECORD_FIELDS = 5


def shard_range(total, rank, world):
    """Contiguous candidate block [lo, hi) of ``rank`` (sizes differ by at most one)."""
    base, extra = divmod(total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def record_width(n_dofs, n_tips):
    return RECORD_FIELDS + n_tips + n_dofs + n_tips + 3 * n_tips + 6


def default_capacity(total, world):
    """Records per rank: the largest shard (⌈total / world⌉), identical on every rank."""
    return -(-int(total) // int(world))


def pack_survivors(capacity, object_id, rank, cand_offset, best_loss, margin, q, comp, target, palm):
    """[capacity + 1, W] float64 buffer; row 0 = header [stored, survived, capacity], rows 1.. =
    surviving candidates in candidate order (the first ``capacity`` of them)."""
    E, T = margin.shape
    D = q.shape[1]
    W = record_width(D, T)
    dev = margin.device
    survive = (margin > 0).all(dim=1)
    all_idx = torch.nonzero(survive).flatten()
    idx = all_idx[:capacity]
    buf = torch.zeros(capacity + 1, W, dtype=torch.float64, device=dev)
    n = idx.numel()
    buf[0, 0] = n
    buf[0, 1] = all_idx.numel()
    buf[0, 2] = capacity
    if n:
        cols = [torch.full((n, 1), float(object_id), dtype=torch.float64, device=dev),
                torch.full((n, 1), float(rank), dtype=torch.float64, device=dev),
                (idx + cand_offset).to(torch.float64).unsqueeze(1),
                best_loss[idx].to(torch.float64).unsqueeze(1),
                torch.ones(n, 1, dtype=torch.float64, device=dev),
                margin[idx].to(torch.float64), q[idx].to(torch.float64), comp[idx].to(torch.float64),
                target[idx].reshape(n, -1).to(torch.float64), palm[idx].to(torch.float64)]
        buf[1:n + 1] = torch.cat(cols, dim=1)
    return buf


def unpack_records(gathered):
    """Concatenates the valid rows of every rank's buffer → [n_total, W]."""
    rows = [g[1:1 + int(g[0, 0])] for g in gathered]
    return torch.cat(rows, dim=0) if rows else gathered[0][1:1]


def overflow(gathered):
    """Per-rank count of survivors that did not fit the buffer (0 everywhere = nothing lost)."""
    return [int(g[0, 1]) - int(g[0, 0]) for g in gathered]


def all_gather_survivors(buf, group=None, return_buffers=False):
    """One collective: every rank receives every rank's fixed-capacity buffer (all ranks must
    pass the same shape — see ``default_capacity``)."""
    world = dist.get_world_size(group)
    out = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(out, buf.contiguous(), group=group)
    return (unpack_records(out), out) if return_buffers else unpack_records(out)


def optimize_sharded(optimizer, gpis, q, target, comp, friction_mu, object_id=0, capacity=None, group=None,
                     shard=True):
    """Each rank optimises its shard of the global candidate arrays (already resident on
    its GPU), then all ranks exchange surviving grasps.  Returns (local results, records).
    ``shard=False`` (config 3, one object per rank): the arrays are this rank's own object's
    candidates, optimised whole; every rank must then hold the same candidate count."""
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    if shard:
        lo, hi = shard_range(q.shape[0], rank, world)
    else:
        lo, hi = 0, q.shape[0]
    palm_all = optimizer.palm_offset
    optimizer.palm_offset = palm_all[lo:hi]
    try:
        res = optimizer.optimize(q[lo:hi], target[lo:hi], comp[lo:hi], friction_mu, gpis, verbose=False)
    finally:
        optimizer.palm_offset = palm_all
    opt_q, opt_comp, opt_target, opt_palm, opt_margin = res
    best = optimizer.best_loss if hasattr(optimizer, "best_loss") else torch.zeros(hi - lo, dtype=torch.float64,
                                                                                  device=q.device)
    cap = capacity or (default_capacity(q.shape[0], world) if shard else q.shape[0])
    buf = pack_survivors(cap, object_id, rank, lo, best, opt_margin, opt_q, opt_comp, opt_target, opt_palm)
    if world == 1:
        return res, unpack_records([buf])
    return res, all_gather_survivors(buf, group)
