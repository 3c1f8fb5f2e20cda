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
3. A template whose other end lies far away -- a same-contig insert longer than the defer span
   (bam.DEFAULT_DEFER_SPAN, half the slack), a mate on another contig, unmapped or absent, whose
   key sorts at its contig's end -- is deferred, as in the one-process stream
   (include/bsdc_io.h bsdc_bam_stream_set_defer): its records go to the spill of the rank whose
   core coordinates (between its boundaries) hold them, its key is registered by the key's owner,
   and the owner cuts its output into pieces at every deferred key (and defers the families that
   may interleave with one).  No record is then foreign to every window.  Phase 2: the parent joins
   the spills into one BAM in file order, and one rank runs the stream over it, cut at the union
   of the deferred keys (bam._stream_step late_splices).
4. The parent assembles the pieces of every rank and of phase 2 in key order, then one BGZF EOF
   block (bam.assemble).  The BAM and the FASTQ pair decompress to the one-process stream's bytes
   (tests/test_ranks.py, with mates on a second contig, unmapped mates and long inserts); only the
   BGZF block boundaries at the seams differ.
5. With deferral off (defer=0) a template whose insert is longer than slack would have its far
   record outside its owner's window: a rank that drops such a record stops at once, and the
   parent reruns the file as one range or raises ForeignRecords (on_foreign).

Every rank's memory is bounded as the one-GPU stream's (about six chunks), and each rank decodes
about 1/N of the records plus 2 * slack positions.  No collective: the ranks exchange nothing but
their spill files and their counts and cut points.

Start-up: neither the parent nor a rank's host stages import torch (the rank processes are plain
multiprocessing spawns).  A rank reports ready at once and creates its engine -- torch, HIP, the
tables -- on a thread of its own (_LazyEngine), while its first job's decoder, reader and planner
already run; the GPU stage takes the engine when it has its first batches.
"""
from __future__ import annotations

import multiprocessing as mp
import os
import threading
import time
import traceback
from typing import List, Optional, Sequence, Tuple

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
    """One rank's part of the file: the one-GPU stream over its window, its own keys only -- or the
    spill's pass (job["late"]: the deferred keys to cut at)."""
    from . import bam
    st, rs = {}, {}
    t0 = time.perf_counter()
    marks: list = []
    try:
        info = bam._stream_step(job["in_bam"], job["fasta"], job["out_bam"], eng, job["prefix"], job["threads"],
                                job["level"], job["fastq"], job["tags"], job["chunk_bytes"], job["slack"],
                                job["batch_bases"], st, job["gpu_bgzf"] and runner is None, None, rng=job["rng"],
                                fragment=job["fragment"], runner=runner, range_stats=rs,
                                owner=(r, job["cuts"], job["flags"]) if job["cuts"] else None, spill=job["spill"],
                                marks=marks, defer=job["defer"], late_splices=job.get("late"),
                                first_key=job.get("first_key"), read_size=job.get("read_size", 8 << 20),
                                regions=True)
    except OSError as e:
        if "foreign record" in str(e):
            return ("foreign", r, str(e))
        raise
    info["seconds"] = round(time.perf_counter() - t0, 4)
    info["marks"] = marks
    rs.pop("spill_tail", None)
    rs.pop("splices_tail", None)
    return ("done", r, info, st, rs)


class _LazyEngine:
    """An engine (or a fleet-style runner) being created on a thread of its own: attribute access
    waits for it; load_reference before it exists is kept and applied once it does.  Lets a rank's
    host stages start while torch loads and HIP initialises (module docstring)."""

    lazy = True

    def __init__(self, make):
        self._ev = threading.Event()
        self._lock = threading.Lock()
        self._obj, self._err, self._ref = None, None, None
        threading.Thread(target=self._init, args=(make,), daemon=True).start()

    def _init(self, make):
        try:
            self._obj = make()
        except BaseException as e:  # noqa: BLE001 -- raised to whoever needs the engine
            self._err = e
        finally:
            self._ev.set()

    def ready(self) -> bool:
        return self._ev.is_set()

    def get(self):
        self._ev.wait()
        if self._err is not None:
            raise RuntimeError("engine creation failed: %s: %s" % (type(self._err).__name__, self._err))
        with self._lock:
            if self._ref is not None:
                ref, self._ref = self._ref, None
                self._obj.load_reference(ref)
        return self._obj

    def load_reference(self, ref):
        with self._lock:
            if not self._ev.is_set():
                self._ref = ref
                return
        self.get().load_reference(ref)

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        return getattr(self.get(), name)


def _make_engine(device: int, runner_spec: Optional[str]):
    if runner_spec is None:
        from .device import Engine
        return Engine(device)
    import importlib
    mod, cls = runner_spec.split(":")
    return getattr(importlib.import_module(mod), cls)(device)


def _rank_server(i: int, device: int, runner_spec: Optional[str], tq, rq):
    """A pool's rank process (spawned: the first thing here to touch its GPU): ready at once, its
    engine or runner created on a thread meanwhile (_LazyEngine), then jobs until None.  Replies
    carry the job's call id."""
    eng = runner = None
    try:
        lazy = _LazyEngine(lambda: _make_engine(device, runner_spec))
        if runner_spec is None:
            eng = lazy
        else:
            runner = lazy
        rq.put(("ready", i, None))
        while True:
            job = tq.get()
            if job is None:
                break
            try:
                rq.put(_run_job(job["rank"], eng, runner, job) + (job["call"],))
            except BaseException as e:  # noqa: BLE001 -- reported to the parent, which raises it
                rq.put(("error", job["rank"], "%s: %s\n%s" % (type(e).__name__, e, traceback.format_exc()), job["call"]))
    except BaseException as e:  # noqa: BLE001
        rq.put(("error", i, "%s: %s\n%s" % (type(e).__name__, e, traceback.format_exc()), None))
    finally:
        try:
            if eng is not None:
                eng.close()
            if runner is not None and hasattr(runner, "close"):
                runner.close()
        except BaseException:  # noqa: BLE001 -- (its creation failed: reported with the job)
            pass


class RankPool:
    """N rank processes, one per device, spawned before this process touches any GPU (spawn
    context), each holding its engine across calls of step5_ranks(pool=...): start it outside a
    timed region, as fleet.Fleet's workers are.  A pool whose rank died is broken: it refuses
    further runs (a dead rank's call may still have replies in flight)."""

    def __init__(self, devices: Sequence[int], runner: Optional[str] = None):
        ctx = mp.get_context("spawn")
        self.rq = ctx.Queue()
        self.tqs = [ctx.Queue() for _ in devices]
        self.procs = [ctx.Process(target=_rank_server, args=(i, int(d), runner, self.tqs[i], self.rq), daemon=True)
                      for i, d in enumerate(devices)]
        for p in self.procs:
            p.start()
        self.n = len(devices)
        self.calls = 0
        self.broken = False
        try:
            for _ in range(self.n):
                m = self.get()
                if m[0] != "ready":
                    raise RuntimeError("rank failed to start: %s" % (m,))
        except BaseException:
            self.close(terminate=True)
            raise

    def get(self):
        """The next rank message; raises (and breaks the pool) if a rank died."""
        import queue
        while True:
            try:
                return self.rq.get(timeout=1.0)
            except queue.Empty:
                dead = [i for i, p in enumerate(self.procs) if not p.is_alive()]
                if dead:
                    self.broken = True
                    raise RuntimeError("rank %d exited (code %s)" % (dead[0], self.procs[dead[0]].exitcode))

    def run(self, jobs: Sequence[dict]) -> list:
        """Jobs 0..k-1 on ranks 0..k-1 (k <= n); their results in order.  A failing or foreign
        rank raises after every rank has answered (the pool stays usable); replies of an earlier
        call (its ranks answered after it raised) are dropped by their call id."""
        if self.broken:
            raise RuntimeError("rank pool is broken (a rank exited); start a new one")
        self.calls += 1
        call = self.calls
        for r, job in enumerate(jobs):
            self.tqs[r].put(dict(job, rank=r, call=call))
        res, bad = {}, None
        while len(res) < len(jobs):
            m = self.get()
            if m[-1] != call:
                continue
            m = m[:-1]
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


def step5_ranks(in_bam: str, fasta: str, out_bam: Optional[str], devices: Sequence[int], prefix: Optional[str] = None,
                threads: int = 0, level: int = 6, fastq: Optional[Tuple[str, str]] = None, tags: bool = True,
                chunk_bytes: Optional[int] = None, slack: Optional[int] = None, batch_bases: Optional[int] = None,
                runner: Optional[str] = None, stats: Optional[dict] = None, gpu_bgzf: bool = False,
                cuts: Optional[list] = None, on_foreign: str = "one", pool: Optional[RankPool] = None,
                defer: Optional[int] = None, read_size: int = 8 << 20) -> dict:
    """Rules convert_Bstrain .. callduplex (main.snake.py:121-164) on a coordinate-sorted BAM by
    len(devices) rank processes (see the module docstring); same file contract as bam.step5_stream.
    runner: "module:Class" of a fleet-style runner (the CPU stand-in of the tests) instead of the
    GPU; cuts: the rank boundaries to use (tests; default plan_cuts).  defer: the span past which a
    template is deferred (default half the slack; 0 = off, when a record no rank can own does what
    on_foreign says -- "one": rerun the file as one range, "raise": ForeignRecords, the caller picks
    another path: cli.py runs fleet.step5_stream_multi).  pool: a started RankPool of at least
    len(devices) ranks to run on (its devices then; default: one is spawned for this call and closed
    after)."""
    import uuid

    import numpy as np

    from . import bam
    if out_bam is None and fastq is None:
        raise ValueError("step5_ranks: no output (out_bam and fastq are both None)")
    chunk_bytes = bam.DEFAULT_CHUNK_BYTES if chunk_bytes is None else chunk_bytes
    slack = bam.DEFAULT_SLACK if slack is None else slack
    dspan = slack // 2 if defer is None else int(defer)
    t0 = time.perf_counter()
    if cuts is None:
        cuts = plan_cuts(in_bam, len(devices), threads, slack)
    t_cut = time.perf_counter() - t0
    hdr = bam.read_bam_header(in_bam)
    pre = bam.read_name_prefix(hdr) if prefix is None else prefix

    tmpdir = os.path.dirname(os.path.abspath(out_bam if out_bam is not None else fastq[0]))
    tag = "%s.rank.%s" % (os.getpid(), uuid.uuid4().hex[:12])

    def paths(t, n, spill):
        return [dict(bam=os.path.join(tmpdir, ".%s.%d.bam" % (t, r)) if out_bam is not None else None,
                     fq=(os.path.join(tmpdir, ".%s.%d.r1.fq.gz" % (t, r)), os.path.join(tmpdir, ".%s.%d.r2.fq.gz" % (t, r)))
                     if fastq is not None else None,
                     spill=os.path.join(tmpdir, ".%s.%d.spill" % (t, r)) if spill else None) for r in range(n)]

    def remove(fr):
        for f in fr:
            for path in ([f["bam"]] if f["bam"] else []) + (list(f["fq"]) if f["fq"] else []) + \
                    ([f["spill"]] if f["spill"] else []):
                if os.path.exists(path):
                    os.unlink(path)

    def first_key(r, cuts):  # the sort key of rank r's first piece (its lower boundary's)
        return (bam.MINKEY, 0, 1) if r == 0 else (cuts[r - 1]["key"][0], cuts[r - 1]["key"][1], 1)

    def run(cuts, pl: "RankPool", ranges, t: str, dsp: int):
        n = len(ranges)
        fr = paths(t, n, dsp > 0)
        jobs = [dict(in_bam=in_bam, fasta=fasta, out_bam=fr[r]["bam"], prefix=pre, threads=threads, level=level,
                     fastq=fr[r]["fq"], tags=tags, chunk_bytes=chunk_bytes, slack=slack, batch_bases=batch_bases,
                     gpu_bgzf=gpu_bgzf, rng=ranges[r], cuts=cuts, flags=bam.OWN_STOP_FOREIGN, spill=fr[r]["spill"],
                     fragment="first" if r == 0 else "next", defer=dsp, first_key=first_key(r, cuts),
                     read_size=read_size)
                for r in range(n)]
        try:
            return pl.run(jobs), fr
        except BaseException:
            remove(fr)  # (every rank of this call has answered: none still writes)
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
    frags, phase2, fr2, spill_bam = [], [], [], None
    n_def = 0
    try:
        t1 = time.perf_counter()
        foreign = 0
        try:
            ranges = windows_of(cuts)
            results, frags = run(cuts, pool, ranges, tag, dspan)
        except ForeignRecords:  # (no fragments are left; only with deferral off)
            if on_foreign == "raise" or not cuts:
                raise
            foreign = 1
            cuts, ranges = [], windows_of([])
            results, frags = run(cuts, pool, ranges, tag, dspan)
        t2 = time.perf_counter()
        # phase 2: the deferred templates of every rank's core share, in file order, through one
        # rank's stream, cut at every rank's deferred keys
        splices = [x[0]["splices"] for x in results if len(x[0]["splices"])]
        spilled = sum(int(x[0].get("spilled_bytes", 0)) for x in results)
        if spilled or splices:
            late = np.unique(np.concatenate(splices), axis=0) if splices else np.zeros((0, 2), np.int64)
            spill_bam = os.path.join(tmpdir, ".%s.spill.bam" % tag)
            n_def = bam.write_spill_bam(spill_bam, hdr, [f["spill"] for f in frags], 1, threads)
            fr2 = paths(tag + "x", 1, False)
            job = dict(in_bam=spill_bam, fasta=fasta, out_bam=fr2[0]["bam"], prefix=pre, threads=threads, level=level,
                       fastq=fr2[0]["fq"], tags=tags, chunk_bytes=chunk_bytes, slack=slack, batch_bases=batch_bases,
                       gpu_bgzf=gpu_bgzf, rng=None, cuts=[], flags=0, spill=None, fragment="next", defer=0,
                       late=late, read_size=read_size)
            try:
                phase2 = pool.run([job])
            except BaseException:
                remove(fr2)
                raise
        t2b = time.perf_counter()
        pieces = []
        for ph, (res, fr) in enumerate(((results, frags), (phase2, fr2))):
            for r, (inf, _, _) in enumerate(res):
                f = fr[r]
                pieces += bam.pieces_of(inf["marks"], [f["bam"]] + (list(f["fq"]) if f["fq"] else [None, None]), ph, r)
        dsts = [out_bam, fastq[0] if fastq else None, fastq[1] if fastq else None]
        for k in range(3):
            if dsts[k] is not None:
                bam.assemble(dsts[k], pieces, k)
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
    info = {"ranks": len(ranges), "cuts_fallback": foreign > 0, "deferred_records": n_def, "records_in": 0,
            "families": 0, "families_emitted": 0, "records_out": 0}
    for inf, st, rs in list(results) + list(phase2):
        for k in ("records_in", "families", "families_emitted", "records_out"):
            info[k] += int(inf.get(k, 0))
    if stats is not None:
        stats.update(cut_s=round(t_cut, 4), pool_start_s=round(t_pool, 4), ranks_s=round(t2 - t1, 4),
                     deferred_s=round(t2b - t2, 4), assemble_s=round(t3 - t2b, 4),
                     rank_records=[int(x[0].get("records_in", 0)) for x in results],
                     rank_read=[int(x[2].get("n", 0)) for x in results],
                     rank_peak_buffered=[int(x[0].get("peak_buffered", 0)) for x in results],
                     rank_seconds=[x[0].get("seconds") for x in results], ranges=ranges)
    return info
