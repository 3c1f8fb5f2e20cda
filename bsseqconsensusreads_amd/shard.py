"""Multi-GPU plumbing of the step: family batches dealt to ranks, no data-path collective.

MI families are independent, so N GPUs are N independent workers: the host cuts the
family stream into contiguous batches balanced by bases (not by family count -- C4's skew), deals
them round-robin to the ranks (one process per GPU, torch.distributed), and gathers the per-batch
outputs back in input order.  The only collectives are the step-time MAX and the counter SUM of
the bench line (8 + 16 bytes) and the host-side object gather of the outputs.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import numpy as np
import torch


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
