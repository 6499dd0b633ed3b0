"""Multi-process path on CPU (gloo, world size 2): candidate sharding and the
fixed-capacity surviving-grasp all-gather."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from compliancedex_amd.distributed import (all_gather_survivors, pack_survivors, record_width, shard_range,
                                           unpack_records)


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
    import numpy as np
    full = np.concatenate(expect)
    for r in range(2):
        assert np.array_equal(res[r], full)
    assert set(full[:, 1]) <= {0.0, 1.0}
