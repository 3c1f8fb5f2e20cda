"""Step 5 over N GPUs of one node with no single front end: N rank processes, each decoding,
computing and encoding its own share of the BAM.

The path is MI families, which are independent.  fleet.step5_stream_multi feeds N
GPU workers from one coordinator that reads, plans and writes the whole file, so on one node its
front end, not the GPUs, sets the pace.  Here the file itself is partitioned, by
template key rather than by record range: in deep data every position is covered by templates,
so no record boundary has all templates before it closed, but the keys (a template's lower
unclipped 5' end, TemplateCoordinate order) leave gaps.

1. The parent (which never touches a GPU) picks N - 1 boundaries X_1 < .. < X_N-1 in key gaps:
   for each nominal split point r * size / N, bam.find_cut (include/bsdc_io.h bsdc_bam_find_cut)
   syncs to the first BGZF block and record boundary after it and takes the first position x on
   that contig, at least 2 * slack on, with no same-contig template key within KEY_GUARD positions
   (a family's keys lie within the tools' jitter of each other, so none straddles x).  It also
   returns where the records at x - slack and at x + slack start.  That reads a few MB per cut.
2. Rank r owns the keys [X_r, X_r+1).  It runs the one-GPU streaming step (bam._stream_step:
   decode, plan, GPU, records, BGZF) over the window from the record at X_r - slack to the one
   at X_r+1 + slack (windows overlap by 2 * slack) and keeps only the records it owns
   (bsdc_bam_stream_set_owner): a template's records near a boundary are read by both ranks and
   kept by one.  It writes a fragment of each output: rank 0 the header and its records, the
   others their records, none an EOF block.
3. Templates whose mate is on another contig or unmapped have keys that sort at their contig's
   end, whatever their records' positions: no window holds them.  Every rank spills those of its
   core share (its own coordinates, between its boundaries) to a file instead of streaming them
   (bsdc_bam_stream_spill), and cuts its chunks so that each holds families of one key contig,
   recording a cut point after the header and after every chunk (BamWriter / FastqWriter
   flush + tell).  Phase 2: the parent joins the spills into one BAM, and each rank runs the
   stream over it, keeping the keys it owns, so the owner of a contig's end forms that contig's
   cross-key families (recording its cut points too).
4. The parent splices the pieces in key order: per contig, the ranks' same-contig pieces in rank
   order, then the contig's cross-key pieces, then one BGZF EOF block.  The BAM and the FASTQ pair
   decompress to the one-process stream's bytes (tests/test_ranks.py, with mates on a second
   contig and unmapped mates too); only the BGZF block boundaries at the seams differ.
5. What remains is a template whose insert is longer than slack, whose far record lies outside its
   owner's window: a rank that drops such a record stops at once.  The parent then reruns the
   file as one range, or raises ForeignRecords for its caller to pick another path (cli.py:
   fleet.step5_stream_multi).

Every rank's memory is bounded as the one-GPU stream's (about six chunks), and each rank decodes
about 1/N of the records plus 2 * slack positions.  No collective: the ranks exchange nothing but
their spill files and their counts and cut points.
"""
from __future__ import annotations

import os
import shutil
import time
import traceback
from typing import List, Optional, Sequence, Tuple

import torch.multiprocessing as tmp

EOF_BLOCK = bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")


def plan_cuts(path: str, n: int, threads: int = 0, slack: Optional[int] = None) -> List[dict]:
    """The rank boundaries (bam.find_cut dicts) that split `path` into at most n key intervals of
    about equal compressed size, in key order; fewer when boundaries coincide (a small file) or
    none exists after a split point."""
    from concurrent.futures import ThreadPoolExecutor

    from . import bam
    sl = bam.DEFAULT_SLACK if slack is None else slack
    size = os.path.getsize(path)
    starts = [size * r // n for r in range(1, n)]
    with ThreadPoolExecutor(max_workers=max(1, min(8, n - 1))) as ex:  # (the C call drops the GIL)
        found = list(ex.map(lambda s: bam.find_cut(path, s, threads, slack=sl), starts))
    cuts = {}
    for c in found:
        if c is not None:
            cuts.setdefault(c["key"], c)
    return [cuts[k] for k in sorted(cuts)]


def windows_of(cuts) -> List[Tuple[int, int, int, int]]:
    """Rank r's record window (start block, offset, end block, offset): from the record at its
    lower boundary - slack to the one at its upper boundary + slack (-1: the first record / the
    end of the file)."""
    lo = [(-1, 0)] + [c["start"] for c in cuts]
    hi = [c["end"] for c in cuts] + [(-1, 0)]
    return [(lo[r][0], lo[r][1], hi[r][0], hi[r][1]) for r in range(len(cuts) + 1)]


def _run_job(r: int, eng, runner, job: dict) -> tuple:
    """One rank's part of the file: the one-GPU stream over its window, its own keys only."""
    from . import bam
    st, rs = {}, {}
    t0 = time.perf_counter()
    marks = [] if job["cuts"] else None
    try:
        info = bam._stream_step(job["in_bam"], job["fasta"], job["out_bam"], eng, job["prefix"], job["threads"],
                                job["level"], job["fastq"], job["tags"], job["chunk_bytes"], job["slack"],
                                job["batch_bases"], st, job["gpu_bgzf"] and runner is None, None, rng=job["rng"],
                                fragment=job["fragment"], runner=runner, range_stats=rs,
                                owner=(r, job["cuts"], job["flags"]) if job["cuts"] else None, spill=job["spill"],
                                marks=marks)
    except OSError as e:
        if "foreign record" in str(e):
            return ("foreign", r, str(e))
        raise
    info["seconds"] = round(time.perf_counter() - t0, 4)
    info["marks"] = marks
    return ("done", r, info, st, rs)


def _rank_server(i: int, device: int, runner_spec: Optional[str], tq, rq):
    """A pool's rank process (spawned: the first thing here to touch its GPU): its engine or
    runner once, then jobs until None."""
    eng = runner = None
    try:
        if runner_spec is None:
            from .device import Engine
            eng = Engine(device)
        else:
            import importlib
            mod, cls = runner_spec.split(":")
            runner = getattr(importlib.import_module(mod), cls)(device)
        rq.put(("ready", i))
        while True:
            job = tq.get()
            if job is None:
                break
            try:
                rq.put(_run_job(job["rank"], eng, runner, job))
            except BaseException as e:  # noqa: BLE001 -- reported to the parent, which raises it
                rq.put(("error", job["rank"], "%s: %s\n%s" % (type(e).__name__, e, traceback.format_exc())))
    except BaseException as e:  # noqa: BLE001
        rq.put(("error", i, "%s: %s\n%s" % (type(e).__name__, e, traceback.format_exc())))
    finally:
        if eng is not None:
            eng.close()
        if runner is not None and hasattr(runner, "close"):
            runner.close()


class RankPool:
    """N rank processes, one per device, spawned before this process touches any GPU (spawn
    context), each holding its engine across calls of step5_ranks(pool=...): start it outside a
    timed region, as fleet.Fleet's workers are."""

    def __init__(self, devices: Sequence[int], runner: Optional[str] = None):
        ctx = tmp.get_context("spawn")
        self.rq = ctx.Queue()
        self.tqs = [ctx.Queue() for _ in devices]
        self.procs = [ctx.Process(target=_rank_server, args=(i, int(d), runner, self.tqs[i], self.rq), daemon=True)
                      for i, d in enumerate(devices)]
        for p in self.procs:
            p.start()
        self.n = len(devices)
        try:
            for _ in range(self.n):
                m = self.get()
                if m[0] != "ready":
                    raise RuntimeError("rank failed to start: %s" % (m,))
        except BaseException:
            self.close(terminate=True)
            raise

    def get(self):
        """The next rank message; raises if a rank died."""
        import queue
        while True:
            try:
                return self.rq.get(timeout=1.0)
            except queue.Empty:
                dead = [i for i, p in enumerate(self.procs) if not p.is_alive()]
                if dead:
                    raise RuntimeError("rank %d exited (code %s)" % (dead[0], self.procs[dead[0]].exitcode))

    def run(self, jobs: Sequence[dict]) -> list:
        """Jobs 0..k-1 on ranks 0..k-1 (k <= n); their results in order.  A failing or foreign
        rank raises after every rank has answered (the pool stays usable)."""
        for r, job in enumerate(jobs):
            self.tqs[r].put(dict(job, rank=r))
        res, bad = {}, None
        while len(res) < len(jobs):
            m = self.get()
            res[m[1]] = m
            if m[0] in ("error", "foreign") and bad is None:
                bad = m
        if bad is not None:
            if bad[0] == "foreign":
                raise ForeignRecords("rank %d: %s" % (bad[1], bad[2]))
            raise RuntimeError("rank %d: %s" % (bad[1], bad[2]))
        return [res[r][2:] for r in range(len(jobs))]

    def close(self, terminate: bool = False):
        for q in self.tqs:
            try:
                q.put(None)
            except Exception:  # noqa: BLE001
                pass
        for p in self.procs:
            if terminate and p.is_alive():
                p.terminate()
            p.join(30)
            if p.is_alive():
                p.kill()
                p.join(5)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close(terminate=exc[0] is not None)


class ForeignRecords(RuntimeError):
    """A rank met a record whose owner never reads it (step5_ranks on_foreign="raise")."""


def _concat(dst: str, parts: Sequence[str]):
    """The fragments in rank order, then one BGZF EOF block."""
    import shutil
    with open(dst, "wb") as out:
        for p in parts:
            with open(p, "rb") as f:
                shutil.copyfileobj(f, out, 1 << 24)
        out.write(EOF_BLOCK)


def _pieces(results, frags, phase2, fr2) -> list:
    """Every rank output's pieces between its cut points (the marks _stream_step records after the
    header and after each chunk), as (key contig, phase, rank, index, paths, starts, ends), in
    output order: each contig's same-contig families (phase 1, ranks in key order), then its
    cross-key families (phase 2, the owner of the contig's end)."""
    out = []
    for phase, (res, fr) in enumerate(((results, frags), (phase2, fr2))):
        for r, (inf, _, _) in enumerate(res):
            f = fr[r]
            ps = [f["bam"], f["fq"][0] if f["fq"] else None, f["fq"][1] if f["fq"] else None]
            prev = [0, 0, 0]
            for i, m in enumerate(inf.get("marks") or []):
                end = [m[0], m[1], m[2]]
                out.append((m[3], phase, r, i, ps, list(prev), end))
                prev = end
            size = [os.path.getsize(p) if p else 0 for p in ps]
            if any(size[k] > prev[k] for k in range(3)):  # (the last mark follows the last chunk)
                raise RuntimeError("rank %d phase %d: bytes after its last cut point" % (r, phase + 1))
    out.sort(key=lambda x: (x[0], x[1], x[2], x[3]))
    return out


def _assemble(dst: str, pieces, k: int):
    """Output file k (0 the BAM, 1 / 2 the FASTQ pair) from its pieces in order, then one EOF block."""
    with open(dst, "wb") as out:
        for p in pieces:
            path, a, b = p[4][k], p[5][k], p[6][k]
            if path is None or b <= a:
                continue
            with open(path, "rb") as f:
                f.seek(a)
                left = b - a
                while left > 0:
                    buf = f.read(min(left, 1 << 24))
                    if not buf:
                        raise RuntimeError("%s: short piece" % path)
                    out.write(buf)
                    left -= len(buf)
        out.write(EOF_BLOCK)


def step5_ranks(in_bam: str, fasta: str, out_bam: Optional[str], devices: Sequence[int], prefix: Optional[str] = None,
                threads: int = 0, level: int = 6, fastq: Optional[Tuple[str, str]] = None, tags: bool = True,
                chunk_bytes: Optional[int] = None, slack: Optional[int] = None, batch_bases: Optional[int] = None,
                runner: Optional[str] = None, stats: Optional[dict] = None, gpu_bgzf: bool = False,
                cuts: Optional[list] = None, on_foreign: str = "one", pool: Optional[RankPool] = None) -> dict:
    """Rules convert_Bstrain .. callduplex (main.snake.py:121-164) on a coordinate-sorted BAM by
    len(devices) rank processes (see the module docstring); same file contract as bam.step5_stream.
    runner: "module:Class" of a fleet-style runner (the CPU stand-in of the tests) instead of the
    GPU; cuts: the rank boundaries to use (tests; default plan_cuts).  on_foreign: what a record
    no rank can own does -- "one": rerun the file as one range (the default), "raise":
    ForeignRecords (the caller picks another path: cli.py runs fleet.step5_stream_multi).  pool: a
    started RankPool of at least len(devices) ranks to run on (its devices then; default: one is
    spawned for this call and closed after)."""
    from . import bam
    chunk_bytes = bam.DEFAULT_CHUNK_BYTES if chunk_bytes is None else chunk_bytes
    slack = bam.DEFAULT_SLACK if slack is None else slack
    t0 = time.perf_counter()
    if cuts is None:
        cuts = plan_cuts(in_bam, len(devices), threads, slack)
    t_cut = time.perf_counter() - t0
    hdr = bam.read_bam_header(in_bam)
    pre = bam.read_name_prefix(hdr) if prefix is None else prefix

    tmpdir = os.path.dirname(os.path.abspath(out_bam if out_bam is not None else fastq[0]))

    def paths(tag, n, spill):
        return [dict(bam=os.path.join(tmpdir, ".%s.%d.bam" % (tag, r)) if out_bam is not None else None,
                     fq=(os.path.join(tmpdir, ".%s.%d.r1.fq.gz" % (tag, r)), os.path.join(tmpdir, ".%s.%d.r2.fq.gz" % (tag, r)))
                     if fastq is not None else None,
                     spill=os.path.join(tmpdir, ".%s.%d.spill" % (tag, r)) if spill else None) for r in range(n)]

    def remove(fr):
        for f in fr:
            for path in ([f["bam"]] if f["bam"] else []) + (list(f["fq"]) if f["fq"] else []) + \
                    ([f["spill"]] if f["spill"] else []):
                if os.path.exists(path):
                    os.unlink(path)

    def run(cuts, pl: "RankPool", in_path: str, ranges, tag: str, phase: int):
        n = len(ranges)
        fr = paths(tag, n, phase == 0 and len(cuts) > 0)
        flags = (bam.OWN_STOP_FOREIGN | bam.OWN_SPILL_CROSS | bam.OWN_CONTIG_CHUNKS) if phase == 0 else \
            bam.OWN_CONTIG_CHUNKS
        jobs = [dict(in_bam=in_path, fasta=fasta, out_bam=fr[r]["bam"], prefix=pre, threads=threads, level=level,
                     fastq=fr[r]["fq"], tags=tags, chunk_bytes=chunk_bytes, slack=slack, batch_bases=batch_bases,
                     gpu_bgzf=gpu_bgzf, rng=ranges[r], cuts=cuts, flags=flags, spill=fr[r]["spill"],
                     fragment="first" if (r == 0 and phase == 0) else "next") for r in range(n)]
        try:
            return pl.run(jobs), fr
        except BaseException:
            remove(fr)  # (every rank has answered: none still writes)
            raise

    own = pool is None
    if own:
        t_p = time.perf_counter()
        pool = RankPool(list(devices)[:len(cuts) + 1], runner)
        t_pool = time.perf_counter() - t_p
    else:
        t_pool = 0.0
        if pool.n < len(cuts) + 1:
            raise ValueError("a pool of %d ranks for %d ranges" % (pool.n, len(cuts) + 1))
    tag = "%s.rank%d" % (os.getpid(), int(time.time() * 1000) & 0xFFFFFF)
    frags, phase2, fr2, spill_bam = [], [], [], None
    try:
        t1 = time.perf_counter()
        foreign = 0
        try:
            ranges = windows_of(cuts)
            results, frags = run(cuts, pool, in_bam, ranges, tag, 0)
        except ForeignRecords:  # (no fragments are left)
            if on_foreign == "raise" or not cuts:
                raise
            foreign = 1
            cuts, ranges = [], windows_of([])
            results, frags = run(cuts, pool, in_bam, ranges, tag, 0)
        t2 = time.perf_counter()
        # phase 2: the templates with a mate on another contig or unmapped, spilled by every rank
        # from its core share, formed into families by the owners of their keys (the rank whose
        # interval holds their contig's end), on one BAM of all the spills
        n_cross = sum(int(x[2].get("spilled", 0)) for x in results)
        if cuts and n_cross:
            spill_bam = os.path.join(tmpdir, ".%s.spill.bam" % tag)
            hw = bam.BamWriter(spill_bam + ".h", hdr, level, None, "first")
            hw.close(threads)
            with open(spill_bam, "wb") as out:
                for part in [spill_bam + ".h"] + [f["spill"] for f in frags]:
                    with open(part, "rb") as f:
                        shutil.copyfileobj(f, out, 1 << 24)
                out.write(EOF_BLOCK)
            os.unlink(spill_bam + ".h")
            phase2, fr2 = run(cuts, pool, spill_bam, [None] * len(ranges), tag + "x", 1)
        t2b = time.perf_counter()
        if not cuts:  # one range: its fragments as they are
            if out_bam is not None:
                _concat(out_bam, [frags[0]["bam"]])
            if fastq is not None:
                for d in range(2):
                    _concat(fastq[d], [frags[0]["fq"][d]])
        else:
            pieces = _pieces(results, frags, phase2, fr2)
            if out_bam is not None:
                _assemble(out_bam, pieces, 0)
            if fastq is not None:
                for d in range(2):
                    _assemble(fastq[d], pieces, 1 + d)
        t3 = time.perf_counter()
    except BaseException:
        if own:
            pool.close(terminate=True)
            own = False
        raise
    finally:
        remove(frags)
        remove(fr2)
        if spill_bam is not None and os.path.exists(spill_bam):
            os.unlink(spill_bam)
        if own:
            pool.close()
    info = {"ranks": len(ranges), "cuts_fallback": foreign > 0, "cross_records": n_cross, "records_in": 0,
            "families": 0, "families_emitted": 0, "records_out": 0}
    for inf, st, rs in list(results) + list(phase2):
        for k in ("records_in", "families", "families_emitted", "records_out"):
            info[k] += int(inf.get(k, 0))
    if stats is not None:
        stats.update(cut_s=round(t_cut, 4), pool_start_s=round(t_pool, 4), ranks_s=round(t2 - t1, 4),
                     cross_s=round(t2b - t2, 4), assemble_s=round(t3 - t2b, 4),
                     rank_records=[int(x[0].get("records_in", 0)) for x in results],
                     rank_read=[int(x[2].get("n", 0)) for x in results],
                     rank_seconds=[x[0].get("seconds") for x in results], ranges=ranges)
    return info
