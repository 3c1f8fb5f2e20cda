"""The N>1 path on CPU: world-size-2 gloo process group over the same shard/deal/reduce/gather
code bench.py and a multi-GPU run use (families shard, no data-path collective)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from bsseqconsensusreads_amd import shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, fam_bases, batch_bases, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        batches = shard.plan_batches(fam_bases, batch_bases)
        mine = {}
        fams = 0
        for i in shard.deal(batches, world, rank):
            a, b = batches[i]
            # stand-in for the per-batch device output: the family ids it covers
            mine[i] = np.arange(a, b, dtype=np.int64)
            fams += b - a
        t, cnt = shard.reduce_step(dist, 0.5 + rank, [fams, 2 * fams], torch.device("cpu"))
        out = shard.gather_in_order(dist, mine, len(batches))
        if rank == 0:
            q.put((t, cnt, np.concatenate(out) if out else np.zeros(0, np.int64)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_family_sharding_gloo(world):
    rng = np.random.default_rng(3)
    fam_bases = rng.integers(150, 8000, size=997)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fam_bases, 20000, q)) for r in range(world)]
    for p in procs:
        p.start()
    t, cnt, order = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert t == 0.5 + (world - 1)                      # step time: MAX over ranks
    assert cnt == [len(fam_bases), 2 * len(fam_bases)]  # counters: SUM over ranks
    assert np.array_equal(order, np.arange(len(fam_bases)))  # gathered in input order


def test_plan_batches_balanced_and_contiguous():
    fb = np.array([5, 5, 5, 100, 1, 1, 1, 1, 30])
    b = shard.plan_batches(fb, 10)
    assert b[0][0] == 0 and b[-1][1] == len(fb)
    assert all(x[1] == y[0] for x, y in zip(b, b[1:]))
    assert all(e > s for s, e in b)
    for s, e in b:  # within budget unless a single family is bigger than it
        assert fb[s:e].sum() <= 10 or e - s == 1
    assert shard.plan_batches(np.zeros(0, np.int64), 10) == []
    assert shard.plan_batches(fb, 0) == [(0, len(fb))]


def test_deal_round_robin():
    b = [(i, i + 1) for i in range(10)]
    got = sorted(i for r in range(4) for i in shard.deal(b, 4, r))
    assert got == list(range(10))
    assert shard.deal(b, 4, 1) == [1, 5, 9]
    with pytest.raises(ValueError):
        shard.deal(b, 4, 4)
