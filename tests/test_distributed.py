"""Multi-process path on CPU (gloo, world size 2): candidate sharding and the
fixed-capacity surviving-grasp all-gather."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import numpy as np

from compliancedex_amd.anneal import PregraspAnnealer, anneal_sharded
from compliancedex_amd.distributed import (all_gather_survivors, default_capacity, optimize_sharded, overflow,
                                           pack_survivors, record_width, shard_range, unpack_records)


def test_shard_range_covers_exactly():
    for total in (0, 1, 7, 4096, 65536 + 3):
        for world in (1, 2, 3, 8):
            spans = [shard_range(total, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1


def _local(rank, E=10, D=16, T=4):
    g = torch.Generator().manual_seed(rank)
    margin = torch.rand(E, T, generator=g, dtype=torch.float64) - 0.2
    return dict(best_loss=torch.rand(E, generator=g, dtype=torch.float64), margin=margin,
                q=torch.rand(E, D, generator=g, dtype=torch.float64), comp=torch.rand(E, T, generator=g, dtype=torch.float64),
                target=torch.rand(E, T, 3, generator=g, dtype=torch.float64),
                palm=torch.rand(E, 6, generator=g, dtype=torch.float64))


def test_pack_unpack_single():
    d = _local(0)
    buf = pack_survivors(8, 3, 0, 100, **d)
    assert buf.shape == (9, record_width(16, 4))
    rec = unpack_records([buf])
    surv = torch.nonzero((d["margin"] > 0).all(1)).flatten()[:8]
    assert rec.shape[0] == surv.numel()
    assert torch.equal(rec[:, 2], (surv + 100).double())
    assert torch.all(rec[:, 0] == 3) and torch.all(rec[:, 4] == 1)
    assert torch.equal(rec[:, 5:9], d["margin"][surv])


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard_range(20, rank, world)
    d = _local(rank)
    buf = pack_survivors(16, 7, rank, lo, **d)
    rec = all_gather_survivors(buf)
    q.put((rank, rec.numpy()))
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_all_gather_survivors_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    expect = []
    for r in range(2):
        d = _local(r)
        lo, _ = shard_range(20, r, 2)
        expect.append(unpack_records([pack_survivors(16, 7, r, lo, **d)]).numpy())
    full = np.concatenate(expect)
    for r in range(2):
        assert np.array_equal(res[r], full)
    assert set(full[:, 1]) <= {0.0, 1.0}


def _unequal_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    d = _local(rank)
    buf = pack_survivors(16 + 4 * rank, 7, rank, 0, **d)  # rank 1's capacity differs: a config-3 run gone wrong
    try:
        all_gather_survivors(buf)
        q.put((rank, "gathered"))
    except ValueError as e:
        q.put((rank, str(e)))
    dist.destroy_process_group()


def test_all_gather_unequal_capacity_fails_on_every_rank():
    """Buffers of different shape must fail loudly on every rank (one all_reduce before the all_gather),
    not hang or scramble the collective."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_unequal_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(2):
        assert "differ across ranks" in res[r] and "rows 17..21" in res[r], res


def test_pack_header_counts_overflow():
    d = _local(0, E=40)
    n_surv = int((d["margin"] > 0).all(1).sum())
    assert n_surv > 3
    buf = pack_survivors(3, 0, 0, 0, **d)
    assert int(buf[0, 0]) == 3 and int(buf[0, 1]) == n_surv and int(buf[0, 2]) == 3
    assert overflow([buf]) == [n_surv - 3]
    assert unpack_records([buf]).shape[0] == 3
    full = pack_survivors(40, 0, 0, 0, **d)
    assert overflow([full]) == [0]


def test_default_capacity_is_rank_independent():
    for total in (1, 21, 4096, 65537):
        for world in (1, 2, 3, 8):
            cap = default_capacity(total, world)
            assert all(cap >= b - a for a, b in (shard_range(total, r, world) for r in range(world)))
            assert cap == max(b - a for a, b in (shard_range(total, r, world) for r in range(world)))


class _ScriptedOpt:
    """Duck-typed inner optimiser whose result depends on each candidate's own row only."""
    num_iters = 30

    def __init__(self, palm):
        self.palm_offset = palm
        self.seen_palm = None

    def optimize(self, q, target, comp, mu, gpis, verbose=False, init_palm=None):
        palm = init_palm if init_palm is not None else self.palm_offset
        self.seen_palm = palm.clone()
        margin = torch.stack([q[:, 0] - 0.3, q[:, 1] - 0.2, q[:, 2] + 1, q[:, 3] + 1], 1)
        self.best_loss = q.sum(1)
        return q + 1, comp * 2, target, palm.clone(), margin


TOTAL = 21  # odd: shards of 11 and 10 candidates


def _global_inputs():
    g = torch.Generator().manual_seed(5)
    f64 = dict(dtype=torch.float64)
    return dict(q=torch.rand(TOTAL, 16, generator=g, **f64), target=torch.rand(TOTAL, 4, 3, generator=g, **f64),
                comp=torch.rand(TOTAL, 4, generator=g, **f64), palm=torch.arange(TOTAL * 6, **f64).view(TOTAL, 6))


def _run_sharded(kind):
    x = _global_inputs()
    if kind == "optimize":
        opt = _ScriptedOpt(x["palm"])
        res, rec = optimize_sharded(opt, None, x["q"], x["target"], x["comp"], 1, object_id=2)
        rank = dist.get_rank() if dist.is_initialized() else 0
        world = dist.get_world_size() if dist.is_initialized() else 1
        lo, hi = shard_range(TOTAL, rank, world)
        assert torch.equal(opt.palm_offset, x["palm"])            # restored after the call
        assert torch.equal(opt.seen_palm, x["palm"][lo:hi])       # the rank's own palm rows
        return rec
    ann = PregraspAnnealer(_ScriptedOpt(x["palm"]), None, q_sigma=0.0, palm_pos_sigma=0.0, palm_ori_sigma=0.0)
    best, rec = anneal_sharded(ann, x["q"], x["target"], x["comp"], x["palm"], outer_steps=1, object_id=4)
    return rec


def _sharded_worker(rank, world, port, q, kind):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, _run_sharded(kind).numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["optimize", "anneal"])
def test_sharded_gloo_world2_equals_world1(kind):
    """optimize_sharded / anneal_sharded over 2 gloo ranks with an odd candidate count (unequal
    shards, equal buffers): every rank gathers exactly the world-1 records (candidate ids are
    global, palm rows the candidate's own)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sharded_worker, args=(r, 2, port, q, kind)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = _run_sharded(kind).numpy()
    assert ref.shape[0] > 3
    x = _global_inputs()
    cand = ref[:, 2].astype(int)
    assert np.array_equal(ref[:, -6:], x["palm"].numpy()[cand])
    for r in range(2):
        # the rank column differs (world 1 has only rank 0); every other field is identical
        assert np.array_equal(np.delete(res[r], 1, axis=1), np.delete(ref, 1, axis=1))
        lo, _ = shard_range(TOTAL, 1, 2)
        assert np.array_equal(res[r][:, 1], (res[r][:, 2] >= lo).astype(float))


def _object_inputs(rank):
    """Rank r's own object (config 3): 11 − r candidates (unequal counts across ranks)."""
    g = torch.Generator().manual_seed(100 + rank)
    E = 11 - rank
    f64 = dict(dtype=torch.float64)
    return dict(q=torch.rand(E, 16, generator=g, **f64), target=torch.rand(E, 4, 3, generator=g, **f64),
                comp=torch.rand(E, 4, generator=g, **f64), palm=torch.rand(E, 6, generator=g, **f64))


def _per_object_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        x = _object_inputs(rank)
        opt = _ScriptedOpt(x["palm"])
        res, rec, bufs = optimize_sharded(opt, None, x["q"], x["target"], x["comp"], 1, object_id=rank, shard=False,
                                          return_buffers=True)
        q.put((rank, rec.numpy(), [tuple(b.shape) for b in bufs], overflow(bufs)))
    finally:
        dist.destroy_process_group()


def test_optimize_sharded_one_object_per_rank_gloo_world2():
    """shard=False (config 3, distributed.py): each rank optimises its own object's candidates — 11
    and 10 here — and the capacity is agreed over ranks (the larger count), so the all_gather buffers
    have one shape; every rank receives exactly the concatenation of the two ranks' own world-1
    records, with nothing lost to overflow."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_per_object_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        r, rec, shapes, ovf = q.get(timeout=120)
        res[r] = (rec, shapes, ovf)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    expect = []
    for r in range(2):
        x = _object_inputs(r)
        opt = _ScriptedOpt(x["palm"])
        out = opt.optimize(x["q"], x["target"], x["comp"], 1, None)
        buf = pack_survivors(11, r, r, 0, opt.best_loss, out[4], out[0], out[1], out[2], out[3])
        expect.append(unpack_records([buf]).numpy())
    full = np.concatenate(expect)
    assert full.shape[0] >= 2 and set(full[:, 0]) == {0.0, 1.0}
    for r in range(2):
        rec, shapes, ovf = res[r]
        assert shapes == [(12, record_width(16, 4))] * 2
        assert ovf == [0, 0]
        assert np.array_equal(rec, full)


@pytest.mark.gpu
@pytest.mark.parametrize("E,cap", [(4096, 4096), (4096, 7), (1, 3), (0, 5), (3000, 1500), (5000, 2100), (2049, 9000),
                                   (1024, 0), (130, 70), (65, 64)])
def test_native_pack_equals_cpu_layout(E, cap):
    """cdx_pack_survivors (the GPU pack: per-tile counts, then the rows — two launches over the chip,
    header counts written on the device, no host sync, no memset) produces bit for bit the buffer of the CPU (torch-ops) layout: survivors in
    candidate order, overflow counted in the header, unused rows zero — also when the buffer was dirty
    before (the kernel zeroes them itself); NaN margins do not survive.  Ragged sizes cross the
    kernel's 64-candidate tiles with the capacity cut inside a tile."""
    d = _local(3, E=E)
    if E:
        d["margin"][0, 0] = float("nan")
    cpu = pack_survivors(cap, 5, 1, 10, **d)
    dg = {k: v.cuda() for k, v in d.items()}
    dirty = torch.full(((cap + 1) * record_width(d["q"].shape[1], d["margin"].shape[1]),), float("nan"),
                       dtype=torch.float64, device="cuda")
    del dirty  # the caching allocator hands the NaN-filled block to the pack's buffer
    gpu = pack_survivors(cap, 5, 1, 10, **dg)
    torch.cuda.synchronize()
    assert torch.equal(gpu.cpu(), cpu)
    assert torch.equal(unpack_records([gpu]).cpu(), unpack_records([cpu]))
