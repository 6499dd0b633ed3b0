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
the local one), so the default capacity is the same on every rank: ⌈total / world⌉ for a sharded
batch, the largest per-rank candidate count (one all_reduce) for one object per rank.

On the GPU the pack is cdx_pack_survivors (two chip-wide launches over 64-candidate tiles: survivor
counts, then each tile's rows at the prefix of the earlier tiles' counts — compaction in candidate
order, header counts written on the device, no host synchronisation); CPU tensors (the gloo tests) take
the same layout through torch ops.  Reading the gathered headers (``unpack_records``) is the one
host synchronisation of the exchange.
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


def _f64(t, shape):
    if t.dtype is torch.float64 and t.is_contiguous() and tuple(t.shape) == tuple(shape):
        return t.detach()  # already the layout the pack reads (no extra dispatch on the exit path)
    return t.detach().to(torch.float64).reshape(shape).contiguous()


def pack_survivors(capacity, object_id, rank, cand_offset, best_loss, margin, q, comp, target, palm):
    """[capacity + 1, W] float64 buffer; row 0 = header [stored, survived, capacity], rows 1.. =
    surviving candidates in candidate order (the first ``capacity`` of them), the rest zero."""
    E, T = margin.shape
    D = q.shape[1]
    W = record_width(D, T)
    dev = margin.device
    capacity = int(capacity)
    buf = torch.empty(capacity + 1, W, dtype=torch.float64, device=dev)
    tgt = target if (target.dim() == 2 and target.is_contiguous()) else target.reshape(E, 3 * T)
    ins = [_f64(margin, (E, T)), _f64(best_loss, (E,)), _f64(q, (E, D)), _f64(comp, (E, T)), _f64(tgt, (E, 3 * T)),
           _f64(palm, (E, 6))]
    if dev.type == "cuda":
        from . import _native as N
        N.check(N.load().cdx_pack_survivors(E, T, D, *(N.ptr(t) for t in ins), float(object_id), float(rank),
                                            int(cand_offset), capacity, N.ptr(buf), N.stream_ptr(dev)),
                "cdx_pack_survivors")
        return buf
    margin, best_loss, q, comp, target, palm = ins
    survive = (margin > 0).all(dim=1)
    pos = torch.cumsum(survive.to(torch.int64), 0) - 1
    keep = survive & (pos < capacity)
    rows = torch.cat([torch.full((E, 1), float(object_id), dtype=torch.float64),
                      torch.full((E, 1), float(rank), dtype=torch.float64),
                      (torch.arange(E, dtype=torch.float64) + cand_offset).unsqueeze(1), best_loss.unsqueeze(1),
                      torch.ones(E, 1, dtype=torch.float64), margin, q, comp, target, palm], dim=1)
    ext = torch.zeros(capacity + 2, W, dtype=torch.float64)  # row capacity + 1 takes the dropped rows
    ext.index_copy_(0, torch.where(keep, pos + 1, torch.full_like(pos, capacity + 1)), rows)
    buf.copy_(ext[:capacity + 1])
    n = survive.sum()
    buf[0, 0] = torch.clamp(n, max=capacity)
    buf[0, 1] = n
    buf[0, 2] = capacity
    return buf


def unpack_records(gathered):
    """Concatenates the valid rows of every rank's buffer → [n_total, W] (one host read of the
    stored counts: the headers of all ranks in one copy)."""
    if len(gathered) == 1:
        g = gathered[0]
        return g[1:1 + int(g[0, 0])]
    counts = torch.stack([g[0, 0] for g in gathered]).tolist()
    rows = [g[1:1 + int(n)] for g, n in zip(gathered, counts)]
    return torch.cat(rows, dim=0)


def overflow(gathered):
    """Per-rank count of survivors that did not fit the buffer (0 everywhere = nothing lost)."""
    return [int(g[0, 1]) - int(g[0, 0]) for g in gathered]


def check_equal_shapes(buf, group=None):
    """Raises ValueError on EVERY rank when the ranks' buffers differ in shape (one all_reduce of
    [rows, cols, −rows, −cols] with MAX): an all_gather of unequal buffers would hang or corrupt
    RCCL's receive buffers instead of failing."""
    dev = buf.device if dist.get_backend(group) == "nccl" else torch.device("cpu")
    r, c = int(buf.shape[0]), int(buf.shape[1])
    t = torch.tensor([r, c, -r, -c], dtype=torch.int64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    hi_r, hi_c, lo_r, lo_c = t.tolist()
    if (hi_r, hi_c, -lo_r, -lo_c) != (r, c, r, c):
        raise ValueError(f"survivor buffers differ across ranks: rows {-lo_r}..{hi_r}, cols {-lo_c}..{hi_c} "
                         f"(this rank {r}x{c}); pass one capacity on every rank (default_capacity / agreed_capacity)")


def all_gather_survivors(buf, group=None, return_buffers=False, check_shape=True):
    """One collective: every rank receives every rank's fixed-capacity buffer (all ranks must
    pass the same shape — see ``default_capacity``).  ``check_shape`` (default) verifies that first
    with one all_reduce (check_equal_shapes); a caller that already checked this shape may skip it."""
    world = dist.get_world_size(group)
    if check_shape and world > 1:
        check_equal_shapes(buf, group)
    out = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(out, buf.contiguous(), group=group)
    return (unpack_records(out), out) if return_buffers else unpack_records(out)


def agreed_capacity(n_local, device, group=None):
    """The largest per-rank candidate count (one all_reduce of a scalar): the common buffer
    capacity when every rank optimises its own object's candidates (``shard=False``)."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return int(n_local)
    dev = device if dist.get_backend(group) == "nccl" else torch.device("cpu")
    t = torch.tensor([int(n_local)], dtype=torch.int64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return int(t.item())


def optimize_sharded(optimizer, gpis, q, target, comp, friction_mu, object_id=0, capacity=None, group=None,
                     shard=True, return_buffers=False):
    """Each rank optimises its shard of the global candidate arrays (already resident on
    its GPU), then all ranks exchange surviving grasps.  Returns (local results, records), plus
    the gathered per-rank buffers when ``return_buffers`` (``overflow(buffers)`` then reports
    survivors that did not fit).  ``shard=False`` (config 3, one object per rank): the arrays are
    this rank's own object's candidates, optimised whole; ranks may hold different counts — the
    capacity is the largest of them (``agreed_capacity``)."""
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
    cap = capacity or (default_capacity(q.shape[0], world) if shard else agreed_capacity(q.shape[0], q.device, group))
    buf = pack_survivors(cap, object_id, rank, lo, best, opt_margin, opt_q, opt_comp, opt_target, opt_palm)
    if world == 1:
        records, bufs = unpack_records([buf]), [buf]
    else:
        records, bufs = all_gather_survivors(buf, group, return_buffers=True)
    return (res, records, bufs) if return_buffers else (res, records)
