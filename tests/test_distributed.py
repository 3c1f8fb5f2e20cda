"""The N>1 path on CPU: world-size 2 and 3 over gloo, through exactly the functions bench.py and
`cli step5 --gpus N` use -- shard.launch (one spawned process per rank, the torch.distributed.run
environment), shard.env_rank / init, plan_batches / deal over a real family plan, reduce_step
(time MAX, counters SUM) and gather_in_order (host gather of per-batch outputs, input order).
SURVEY.md 8e: families shard with no data-path collective."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from bsseqconsensusreads_amd import batch, shard, synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _worker(out_path, n_fam, budget):
    """What a rank of `cli step5 --gpus N` does, with the device step replaced by the batch's
    family ids (the host side is the real one: the plan every rank builds identically)."""
    import torch
    rank, world, local = shard.env_rank()
    dist = shard.init("gloo")
    try:
        s = synth.generate("C2", n_fam, seed=3, device="cpu", genome_len=100_000)
        plan = batch.plan_families(s.raw, "full", s.ref)
        ranges = shard.plan_batches(plan.fam_bases(), budget)
        mine = {}
        fams = 0
        for i in shard.deal(ranges, world, rank):
            a, b = ranges[i]
            fb = batch.materialize(plan, a, b)
            mine[i] = fb.src.copy()  # stand-in for the batch's device output: its records
            fams += b - a
        t, cnt = shard.reduce_step(dist, 0.5 + rank, [fams, 2 * fams], torch.device("cpu"))
        out = shard.gather_in_order(dist, mine, len(ranges))
        if rank == 0:
            with open(out_path, "w") as fh:
                json.dump({"t": t, "cnt": cnt, "src": np.concatenate(out).tolist(), "world": world,
                           "n_ranges": len(ranges), "plan_src": plan.order.tolist(), "n_fam": plan.n_fam}, fh)
    finally:
        if dist is not None:
            dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_launch_plan_deal_reduce_gather(world, tmp_path):
    out = str(tmp_path / "r0.json")
    assert shard.launch(world, _worker, (out, 300, 3000)) == 0
    r = json.load(open(out))
    assert r["world"] == world and r["n_ranges"] > world
    assert r["t"] == 0.5 + (world - 1)                       # step time: MAX over ranks
    n_fam = r["n_fam"]
    assert r["cnt"] == [n_fam, 2 * n_fam] and n_fam >= 300  # counters: SUM over ranks
    assert r["src"] == r["plan_src"]                        # batches gathered back in plan order


def _failing(msg):
    raise RuntimeError(msg)


def test_launch_reports_rank_failure():
    assert shard.launch(2, _failing, ("no GPU here",)) == 1


def test_bench_spawns_ranks_and_fails_cleanly_without_gpu():
    """`bench.py --gpus 2` with no launcher spawns 2 ranks itself; without a GPU each rank fails
    with one line and the bench exits non-zero (the parent never touches the GPU)."""
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0",
                        "--cpu-sample", "0"], capture_output=True, text=True, timeout=300,
                       env={k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")})
    assert p.returncode != 0
    assert "rank 0/2" in p.stderr and "rank 1/2" in p.stderr, p.stderr[-2000:]
    q = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], capture_output=True,
                       text=True, timeout=300, env=dict(os.environ, WORLD_SIZE="1"))
    assert q.returncode == 2 and "--gpus 2 but WORLD_SIZE=1" in q.stderr


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
