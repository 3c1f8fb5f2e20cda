"""Rehearsal of `bench.py --gpus N` on a one-GPU box: N spawned ranks run bench.run exactly as the
8-GPU driver run does (shard.launch before any GPU call, each rank its own seeded families, barrier
+ synchronize around the K timed steps, MAX time / SUM families over the ranks, rank 0's JSON line),
except that every rank uses device 0 and the process group is gloo: RCCL refuses two ranks on one
GPU.  So it exercises everything of the N-rank bench but the RCCL transport itself.

Usage (GPU box): python profiles/rehearse_bench_ranks.py --ranks 2 -- --families 200000 --steps 5
(the arguments after -- are bench.py's; --gpus is set to --ranks)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _rank(argv):
    # a spawned rank: nothing has touched the GPU yet.  Every rank on device 0, gloo collectives
    # (the bench's two: barrier and the time / counter all_reduce, moved to host tensors)
    os.environ["LOCAL_RANK"] = "0"
    import torch

    import bench
    from bsseqconsensusreads_amd import shard
    init0, reduce0 = shard.init, shard.reduce_step
    shard.init = lambda backend, device=None: init0("gloo")
    shard.reduce_step = lambda dist, t, c, device: reduce0(dist, t, c, torch.device("cpu"))
    bench.run(bench.parse(argv))
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=2)
    ap.add_argument("bench_args", nargs=argparse.REMAINDER)
    a = ap.parse_args()
    rest = [x for x in a.bench_args if x != "--"]
    from bsseqconsensusreads_amd import shard
    return shard.launch(a.ranks, _rank, (["--gpus", str(a.ranks)] + rest,))


if __name__ == "__main__":
    sys.exit(main())
