"""Multi-GPU plumbing of the step: family batches dealt to ranks, no data-path collective.

MI families are independent, so N GPUs are N independent workers: the host cuts the
family stream into contiguous batches balanced by bases (not by family count -- C4's skew), deals
them round-robin to the ranks (one process per GPU, torch.distributed), and gathers the per-batch
outputs back in input order.  The only collectives are the step-time MAX and the counter SUM of
the bench line (8 + 16 bytes) and the host-side object gather of the outputs.

``launch`` starts the ranks itself (spawn) when no external launcher did, so `bench.py --gpus N`
and `cli step5 --gpus N` run one process per GPU either way.
"""
from __future__ import annotations

import os
import socket
import sys
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np


def plan_batches(fam_bases: np.ndarray, batch_bases: int) -> List[Tuple[int, int]]:
    """Contiguous family ranges [start, end) of about `batch_bases` bases each (never empty,
    never splitting a family; a family larger than batch_bases is a batch of its own)."""
    fam_bases = np.asarray(fam_bases, dtype=np.int64)
    n = fam_bases.shape[0]
    if n == 0:
        return []
    if batch_bases <= 0:
        return [(0, n)]
    cs = np.cumsum(fam_bases)
    out = []
    start, base = 0, 0
    while start < n:
        # last family whose running total stays within the budget (at least one family)
        end = int(np.searchsorted(cs, base + batch_bases, side="right"))
        end = max(end, start + 1)
        out.append((start, end))
        base = int(cs[end - 1])
        start = end
    return out


def deal(batches: Sequence[Tuple[int, int]], world: int, rank: int) -> List[int]:
    """Indices of the batches rank `rank` owns: round-robin over the batch list."""
    if not 0 <= rank < world:
        raise ValueError("rank %d outside world of %d" % (rank, world))
    return list(range(rank, len(batches), world))


def reduce_step(dist, elapsed_s: float, counters: Sequence[int], device) -> Tuple[float, List[int]]:
    """Bench reduction: step time MAX over ranks, counters SUM over ranks.  `dist` None = one rank."""
    import torch
    t = torch.tensor([float(elapsed_s)], dtype=torch.float64, device=device)
    c = torch.tensor([int(x) for x in counters], dtype=torch.int64, device=device)
    if dist is not None:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(c, op=dist.ReduceOp.SUM)
    return float(t[0]), [int(x) for x in c.tolist()]


def gather_in_order(dist, mine: Dict[int, object], n_batches: int, dst: int = 0):
    """Host gather: every rank's {batch index: output} -> the list of outputs in batch order on
    rank `dst` (None elsewhere).  Outputs are host objects (numpy arrays), moved as pickles over
    the process group -- this is the host-side gather of SURVEY.md 8e, not a device collective."""
    if dist is None:
        return [mine[i] for i in range(n_batches)]
    world = dist.get_world_size()
    got = [None] * world if dist.get_rank() == dst else None
    dist.gather_object(mine, got, dst=dst)
    if dist.get_rank() != dst:
        return None
    merged: Dict[int, object] = {}
    for part in got:
        for k, v in part.items():
            if k in merged:
                raise RuntimeError("batch %d produced by two ranks" % k)
            merged[k] = v
    missing = [i for i in range(n_batches) if i not in merged]
    if missing:
        raise RuntimeError("batches %s produced by no rank" % missing[:8])
    return [merged[i] for i in range(n_batches)]


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank_main(rank: int, world: int, port: int, fn: Callable, args: tuple):
    # runs in a fresh (spawned) interpreter: nothing has touched the GPU yet
    os.environ.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                       "LOCAL_WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    try:
        rc = fn(*args)
    except Exception as e:  # noqa: BLE001 -- one line per failing rank, non-zero exit
        print("rank %d/%d: %s: %s" % (rank, world, type(e).__name__, e), file=sys.stderr, flush=True)
        sys.exit(1)
    if rc:
        sys.exit(int(rc))


def launch(world: int, fn: Callable, args: tuple = ()) -> int:
    """One process per GPU without an external launcher: `world` spawned ranks run fn(*args) with
    RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set as torch.distributed.run sets them.  The caller
    must not have touched the GPU (spawn, never fork or exec from a GPU process).  Returns the
    first non-zero exit code of the ranks (0 when all succeed)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    port = free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, fn, args)) for r in range(world)]
    for p in procs:
        p.start()
    code = 0
    for p in procs:
        p.join()
        if p.exitcode and not code:
            code = p.exitcode if p.exitcode > 0 else 128 - p.exitcode
    return code


def env_rank() -> Tuple[int, int, int]:
    """(rank, world, local rank) from the torch.distributed.run environment (1 rank without it)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(backend: str, device=None):
    """torch.distributed over the environment's rendezvous (127.0.0.1); None for one rank."""
    rank, world, _ = env_rank()
    if world <= 1:
        return None
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if backend == "nccl" and device is not None:
        dist.init_process_group(backend, device_id=device)
    else:
        dist.init_process_group(backend)
    return dist
