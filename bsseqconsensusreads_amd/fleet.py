"""Step 5 over N GPUs of one node, streaming: one reader, N GPU workers, one ordered writer.

MI families are independent, so the GPUs never talk to each other.  This process
(the coordinator) never touches a GPU.  It spawns one worker process per device, then runs the
one-GPU stream's front end (bam.step5_stream): a decoder thread reads the coordinate-sorted BAM
once, in bounded chunks (bam.stream_bam), and a planner thread forms each chunk's families
(batch.plan_families, the fgbio TemplateCoordinate runs).  The coordinator cuts every chunk's
families into device batches (pipeline.plan_ranges), builds each batch (C++ materialize) and hands
it to the least-loaded worker through shared memory: arrays travel as torch.multiprocessing
named shared-memory segments, pooled and reused on both sides (SegmentPool): materialize writes
the family images straight into a coordinator segment, the rest of the batch is copied into
another, and only names and offsets are pickled (no process-group traffic).  A worker uploads
the batch to its GPU, runs the kernels (libbsdc, the same launch as one GPU) and fetches the
consensus arrays into a segment of its own, which the coordinator reads in place and releases
once the chunk is written.  A collector thread puts the batches back in input order
and a writer thread turns each complete chunk into records and appends them to the BAM / FASTQ
(bam.duplex_records, BamWriter, FastqWriter): the output is byte-identical to the one-GPU stream.

Memory is bounded whatever the input size: at most `inflight` batches per worker, and the
decoder / planner / writer hand-offs hold one chunk each (reference: the 100 GB note of
README.md:83 and tool 2's whole-file dict, tools/2.extend_gap.py:155-178).

A chunk whose tool-2 extension partners straddle its families (plan.split_ext: inconsistent mate
fields) goes to one worker whole, which runs pipeline.run_step5's two-launch fallback on it.

Workers run a pluggable runner (``runner``: "module:Class"); the default is GpuRunner (libbsdc on
the worker's device).  tests/fleet_standin.py is a CPU stand-in that computes the same arrays with
oracle/, so the whole multi-process path (spawn, chunks, shared memory, order, writer) is tested
on CPU.
"""
from __future__ import annotations

import ctypes
import dataclasses
import importlib
import os
import queue
import threading
import time
import traceback
from multiprocessing import shared_memory
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch.multiprocessing as tmp

from . import records as R

_SMALL = 4096  # arrays below this many bytes travel pickled with the message
_ALIGN = 64


# ------------------------------------------------------------------------------------------
# shared memory: named segments, reused
# ------------------------------------------------------------------------------------------
class SegmentPool:
    """Named shared-memory segments (multiprocessing.shared_memory) owned by this process and
    reused: take() the smallest free segment that fits (or a new one), give() it back once the
    other side has let go of it.  A message's large arrays travel in one segment, so steady state
    allocates nothing and faults no fresh pages (a fresh share_memory_() tensor per array cost as
    much as the copy into it).  close() unlinks every segment."""

    MIN = 16 << 20

    def __init__(self, tag: str, keep: int = 8, pinner: Optional["HostPinner"] = None,
                 on_drop=None):
        self.prefix = "bsdc%d_%s_%x" % (os.getpid(), tag, id(self) & 0xFFFFFF)
        self.pinner = pinner  # (a GPU worker's: its segments are page-locked for DMA)
        self.segs: Dict[str, "shared_memory.SharedMemory"] = {}
        self.free: List[str] = []
        self.keep = keep
        # on_drop(name): a segment was unlinked -- the other side unmaps (and unpins) its view of it
        # (SegmentViews.forget), so neither side's mappings grow over a run
        self.on_drop = on_drop
        self.n = 0
        self.created_bytes = 0  # (stats: fresh segments fault their pages in on first touch)
        self.closed = False
        self.lock = threading.Lock()

    def take(self, nbytes: int) -> str:
        with self.lock:
            fit = [x for x in self.free if self.segs[x].size >= nbytes]
            if fit:
                name = min(fit, key=lambda x: self.segs[x].size)
                self.free.remove(name)
                return name
            name = "%s_%d" % (self.prefix, self.n)
            self.n += 1
        shm = shared_memory.SharedMemory(name=name, create=True, size=max(int(nbytes * 1.25) + _ALIGN, self.MIN))
        if self.pinner is not None:
            self.pinner.pin(shm)
        with self.lock:
            self.segs[name] = shm
            self.created_bytes += shm.size
        return name

    def prefill(self, count: int, size: int, threads: int = 4) -> threading.Thread:
        """Create `count` free segments of `size` bytes and fault their pages in, on a background
        thread (a fresh shared page costs a fault on first touch: ~1 GB/s, several times the copy
        into it).  take() meanwhile creates what it needs itself.  The prefilled segments count
        towards `keep`: give() trims the free list only beyond them, so steady state reuses them
        instead of dropping and re-creating segments."""
        with self.lock:
            self.keep += count

        def run():
            for _ in range(count):
                with self.lock:
                    if self.closed:
                        return
                    name = "%s_%d" % (self.prefix, self.n)
                    self.n += 1
                shm = shared_memory.SharedMemory(name=name, create=True, size=max(int(size), self.MIN))
                _populate(shm, threads)
                if self.pinner is not None:
                    self.pinner.pin(shm)
                with self.lock:
                    if not self.closed:
                        self.segs[name] = shm
                        self.created_bytes += shm.size
                        self.free.append(name)
                        continue
                self._drop(shm)  # (the pool closed meanwhile)
        t = threading.Thread(target=run, daemon=True)
        t.start()
        return t

    def give(self, name: Optional[str]):
        if name is None:
            return
        with self.lock:
            if name not in self.segs:
                return
            self.free.append(name)
            while len(self.free) > self.keep:  # the smallest free ones go
                x = min(self.free, key=lambda y: self.segs[y].size)
                self.free.remove(x)
                self._drop(self.segs.pop(x))
                if self.on_drop is not None:
                    self.on_drop(x)

    def buf(self, name: str) -> memoryview:
        return self.segs[name].buf

    def owns(self, a: np.ndarray) -> Optional[Tuple[str, int]]:
        """(segment, byte offset) of an array that lies in one of this pool's segments."""
        if a.nbytes == 0:
            return None
        p = a.__array_interface__["data"][0]
        with self.lock:
            for name, shm in self.segs.items():
                b = np.frombuffer(shm.buf, np.uint8).__array_interface__["data"][0]
                if b <= p and p + a.nbytes <= b + shm.size:
                    return name, p - b
        return None

    def _drop(self, shm):
        if self.pinner is not None:
            self.pinner.unpin(shm)
        _close(shm, unlink=True)

    def close(self):
        with self.lock:
            self.closed = True
            segs, self.segs, self.free = self.segs, {}, []
        for shm in segs.values():
            self._drop(shm)


_LINGER: list = []  # segments closed while numpy views still mapped them
_MADV_POPULATE_WRITE = 23  # Linux >= 5.14


def _populate(shm, threads: int = 4):
    """Fault a fresh segment's pages in (madvise MADV_POPULATE_WRITE over `threads` slices; one
    write per page where the kernel lacks it)."""
    a = np.frombuffer(shm.buf, np.uint8)
    n = a.shape[0]
    if n == 0:
        return
    try:
        libc = ctypes.CDLL(None, use_errno=True)
        libc.madvise.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        base = a.ctypes.data
        step = -(-n // max(1, threads) // 4096) * 4096
        rcs: List[int] = []

        def one(o):
            rcs.append(libc.madvise(base + o, min(step, n - o), _MADV_POPULATE_WRITE))
        ts = [threading.Thread(target=one, args=(o,)) for o in range(0, n, step)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        if all(r == 0 for r in rcs):
            return
    except (OSError, AttributeError):
        pass
    a[::4096] = 0


def _close(shm, unlink: bool):
    try:
        shm.close()
    except BufferError:  # numpy views still map it: the mapping goes with the views / the process
        _LINGER.append(shm)
    if unlink:
        try:
            shm.unlink()
        except FileNotFoundError:
            pass


class SegmentViews:
    """The other side's segments, opened once by name and kept (no remapping per message)."""

    def __init__(self, pinner: Optional["HostPinner"] = None):
        self.open: Dict[str, "shared_memory.SharedMemory"] = {}
        self.pinner = pinner

    def buf(self, name: str) -> memoryview:
        shm = self.open.get(name)
        if shm is None:
            # (spawned workers share the coordinator's resource tracker, so attaching registers
            # nothing new, and a segment left behind by a dead process is still unlinked at exit)
            shm = shared_memory.SharedMemory(name=name)
            if self.pinner is not None:
                self.pinner.pin(shm)
            self.open[name] = shm
        return shm.buf

    def forget(self, name: str):
        """The owner dropped segment `name`: unmap (and unpin) this side's view of it."""
        shm = self.open.pop(name, None)
        if shm is not None:
            if self.pinner is not None:
                self.pinner.unpin(shm)
            _close(shm, unlink=False)

    def close(self):
        for shm in self.open.values():
            if self.pinner is not None:
                self.pinner.unpin(shm)
            _close(shm, unlink=False)
        self.open = {}


class HostPinner:
    """Page-locks a GPU worker's mappings of the shared segments (libbsdc bsdc_host_register), so a
    batch's arrays upload and its outputs come back by DMA straight from / into the segments; a
    pageable copy goes through the runtime's staging buffers at a fraction of the rate, on the
    worker's CPU.  Best effort: a mapping the runtime refuses stays pageable."""

    def __init__(self, device: int):
        from . import _lib
        self.lib = _lib.load()
        self.device = device
        self.done: Dict[int, int] = {}
        self.lock = threading.Lock()

    def pin(self, shm):
        ptr = np.frombuffer(shm.buf, np.uint8).ctypes.data
        with self.lock:
            if ptr in self.done:
                return
            if self.lib.bsdc_host_register(self.device, ptr, shm.size) == 0:
                self.done[ptr] = shm.size

    def unpin(self, shm):
        try:
            ptr = np.frombuffer(shm.buf, np.uint8).ctypes.data
        except (TypeError, ValueError):  # (already closed)
            return
        with self.lock:
            if self.done.pop(ptr, None) is not None:
                self.lib.bsdc_host_unregister(self.device, ptr)


def pack(obj, pool: Optional[SegmentPool] = None):
    """obj (dataclass / dict / list of numpy arrays, StringTables, scalars) -> (a picklable tree,
    the segments it uses).  Arrays that already lie in one of `pool`'s segments (family images
    materialized there, outputs fetched there) travel by reference; the others are copied into one
    segment taken from `pool`.  The receiver reads them in place; the segments go back to `pool`
    once it is done (the sender's bookkeeping)."""
    big: List[np.ndarray] = []

    def collect(o):
        from .bam import StringTable
        if isinstance(o, np.ndarray):
            if o.nbytes >= _SMALL:
                big.append(o)
        elif isinstance(o, StringTable):
            collect(o.buf)
            collect(o.off)
        elif dataclasses.is_dataclass(o) and not isinstance(o, type):
            for f in dataclasses.fields(o):
                collect(getattr(o, f.name))
        elif isinstance(o, dict):
            for v in o.values():
                collect(v)
        elif isinstance(o, (list, tuple)):
            for v in o:
                collect(v)
    collect(obj)
    place: Dict[int, Tuple[str, int]] = {}
    need = 0
    for a in big:
        loc = pool.owns(a) if pool is not None and a.flags.c_contiguous else None
        if loc is not None:
            place[id(a)] = loc
        else:
            need += (a.nbytes + _ALIGN - 1) // _ALIGN * _ALIGN
    seg = None
    if need:
        if pool is None:
            raise ValueError("pack: large arrays need a segment pool")
        seg = pool.take(need)
        buf = np.frombuffer(pool.buf(seg), np.uint8)
        o = 0
        for a in big:
            if id(a) in place:
                continue
            np.copyto(buf[o:o + a.nbytes], np.ascontiguousarray(a).reshape(-1).view(np.uint8))
            place[id(a)] = (seg, o)
            o += (a.nbytes + _ALIGN - 1) // _ALIGN * _ALIGN

    def tree(o):
        from .bam import StringTable
        if isinstance(o, np.ndarray):
            if o.nbytes < _SMALL:  # (a copy: the queue pickles it later, and o may lie in a reused segment)
                return ("np", np.array(o))
            name, off = place[id(o)]
            return ("sm", name, off, o.dtype.str, o.shape)
        if isinstance(o, StringTable):
            return ("st", tree(o.buf), tree(o.off), o.as_str)
        if dataclasses.is_dataclass(o) and not isinstance(o, type):
            return ("dc", type(o), {f.name: tree(getattr(o, f.name)) for f in dataclasses.fields(o)})
        if isinstance(o, dict):
            return ("di", {k: tree(v) for k, v in o.items()})
        if isinstance(o, (list, tuple)) and any(isinstance(x, np.ndarray) for x in o):
            return ("li", [tree(x) for x in o])
        return ("v", o)
    return tree(obj), sorted({v[0] for v in place.values()})


def unpack(tree, views: Optional[SegmentViews] = None, pool: Optional[SegmentPool] = None):
    """The inverse of pack: numpy views of the named segments (opened through `views`, or this
    process's own `pool`)."""
    from .bam import StringTable
    kind = tree[0]
    if kind == "np":
        return tree[1]
    if kind == "sm":
        _, name, off, dt, shape = tree
        buf = pool.buf(name) if pool is not None and name in pool.segs else views.buf(name)
        dt = np.dtype(dt)
        n = int(np.prod(shape, dtype=np.int64)) if len(shape) else 1
        return np.frombuffer(buf, dt, count=n, offset=off).reshape(shape)
    if kind == "st":
        return StringTable(unpack(tree[1], views, pool), unpack(tree[2], views, pool), tree[3])
    if kind == "dc":
        return tree[1](**{k: unpack(v, views, pool) for k, v in tree[2].items()})
    if kind == "di":
        return {k: unpack(v, views, pool) for k, v in tree[1].items()}
    if kind == "li":
        return [unpack(x, views, pool) for x in tree[1]]
    return tree[1]


# ------------------------------------------------------------------------------------------
# workers
# ------------------------------------------------------------------------------------------
class GpuRunner:
    """A worker's compute: libbsdc on one device (device.Engine)."""

    needs_raw = False

    def __init__(self, device: int):
        from .device import Engine
        self.eng = Engine(device)

    def load_reference(self, ref):
        self.eng.load_reference(ref)

    def run_batch(self, fb, mode: int, tags: bool, raw_sub=None, alloc=None) -> dict:
        """alloc(nbytes) -> a uint8 array the outputs are fetched into (a shared segment)."""
        from ._lib import MODE_TAGS
        db = self.eng.upload(fb, tags=tags)
        self.eng.run(db, mode | (MODE_TAGS if tags else 0))
        return db.fetch(alloc)

    def run_chunk(self, raw, tags: bool, batch_bases):
        from . import pipeline
        return pipeline.run_step5(self.eng, raw, tags=tags, batch_bases=batch_bases)[0]

    def close(self):
        self.eng.close()


def _make_runner(spec: Optional[str], device: int):
    if spec is None:
        return GpuRunner(device)
    mod, cls = spec.split(":")
    return getattr(importlib.import_module(mod), cls)(device)


def _worker(wid: int, device: int, runner_spec: Optional[str], tq, rq):
    """One GPU worker (a spawned process: it is the first thing here to touch the GPU).  Batches
    arrive as views of the coordinator's segments; outputs are fetched into this worker's own
    segments and travel back by name; the coordinator releases them once their chunk is written."""
    runner = None
    pinner = HostPinner(device) if runner_spec is None else None  # (the GPU runner only)
    pool = SegmentPool("w%d" % wid, pinner=pinner, on_drop=lambda name: rq.put(("forget", wid, name)))
    views = SegmentViews(pinner)
    taken: List[str] = []  # the segments alloc() handed out for the current batch

    def alloc(nbytes: int):
        if pool.n == 0:  # the first output: room for as many more, faulted in meanwhile
            pool.prefill(4, int(1.25 * nbytes) + 4096)
        name = pool.take(nbytes)
        taken.append(name)
        return np.frombuffer(pool.buf(name), np.uint8, count=nbytes)

    def unused(segs):
        """Give back the alloc() segments the packed result does not refer to (a tiny
        batch's outputs all travel pickled, so its fetch segment is never released otherwise)."""
        for name in taken:
            if name not in segs:
                pool.give(name)
        taken.clear()
    try:
        runner = _make_runner(runner_spec, device)
        rq.put(("ready", wid, bool(getattr(runner, "needs_raw", False))))
        while True:
            msg = tq.get()
            if msg is None:
                break
            kind = msg[0]
            if kind == "release":
                pool.give(msg[1])
            elif kind == "forget":  # the coordinator dropped one of its segments
                views.forget(msg[1])
            elif kind == "drop":  # the coordinator's run is over: unmap its segments
                views.close()
            elif kind == "ref":
                runner.load_reference(unpack(msg[1], views))
            elif kind == "batch":
                _, key, fb_t, mode, tags, raw_t = msg
                t0 = time.perf_counter()
                fb = unpack(fb_t, views)
                raw_sub = unpack(raw_t, views) if raw_t is not None else None
                if isinstance(runner, GpuRunner):
                    out = runner.run_batch(fb, mode, tags, raw_sub, alloc=alloc)
                else:
                    out = runner.run_batch(fb, mode, tags, raw_sub)
                del fb, raw_sub, fb_t, raw_t
                t1 = time.perf_counter()
                tree, segs = pack(out, pool)
                unused(segs)
                rq.put(("batch", wid, key, tree, segs,
                        {"worker_run": t1 - t0, "worker_pack": time.perf_counter() - t1}))
            elif kind == "chunk":
                _, key, raw_t, tags, batch_bases = msg
                cons = runner.run_chunk(unpack(raw_t, views), tags, batch_bases)
                del raw_t
                tree, segs = pack(cons, pool)
                unused(segs)
                rq.put(("chunk", wid, key, tree, segs, {}))
    except BaseException as e:  # noqa: BLE001 -- reported to the coordinator, which raises it
        rq.put(("error", wid, "%s: %s\n%s" % (type(e).__name__, e, traceback.format_exc())))
        # stay until the coordinator ends the fleet: its segments unlinked now would leave the
        # results it has not opened yet unreadable
        try:
            while tq.get(timeout=600) is not None:
                pass
        except Exception:  # noqa: BLE001
            pass
    finally:
        if runner is not None:
            try:
                runner.close()
            except Exception:  # noqa: BLE001
                pass
        views.close()
        pool.close()


class Fleet:
    """N worker processes, spawned before this process touches any GPU (spawn context: a fresh
    interpreter per worker; nothing is forked or exec'd from a GPU process)."""

    def __init__(self, devices: Sequence[int], runner: Optional[str] = None, inflight: int = 2):
        ctx = tmp.get_context("spawn")
        self.rq = ctx.Queue()
        self.tqs = [ctx.Queue() for _ in devices]
        self.procs = [ctx.Process(target=_worker, args=(i, int(d), runner, self.tqs[i], self.rq), daemon=True)
                      for i, d in enumerate(devices)]
        for p in self.procs:
            p.start()
        self.n = len(devices)
        self.load = [0] * self.n  # jobs in flight per worker (submit: dealer thread, done: collector)
        self._load_lock = threading.Lock()
        self.slots_total = max(1, inflight) * self.n
        self.slots = threading.Semaphore(self.slots_total)
        self.needs_raw = False
        try:
            for _ in range(self.n):
                m = self.get()
                if m[0] != "ready":
                    raise RuntimeError("fleet worker failed to start: %s" % (m,))
                self.needs_raw |= m[2]
        except BaseException:
            self.close(timeout=30.0)
            raise

    def get(self, timeout: Optional[float] = None):
        """The next worker message (None after `timeout` seconds without one); raises if a worker
        reported an error or died."""
        t0 = time.time()
        while True:
            try:
                m = self.rq.get(timeout=1.0 if timeout is None else min(1.0, timeout))
            except queue.Empty:
                dead = [i for i, p in enumerate(self.procs) if not p.is_alive()]
                if dead:
                    raise RuntimeError("fleet worker %d exited (code %s)" % (dead[0], self.procs[dead[0]].exitcode))
                if timeout is not None and time.time() - t0 >= timeout:
                    return None
                continue
            if m[0] == "error":
                raise RuntimeError("fleet worker %d: %s" % (m[1], m[2]))
            return m

    def broadcast(self, msg):
        for q in self.tqs:
            q.put(msg)

    def submit(self, msg, stop: Optional[threading.Event] = None) -> int:
        """Queue a job on the least-loaded worker (blocks while every worker holds `inflight`);
        -1 when `stop` is set first."""
        while not self.slots.acquire(timeout=0.5):
            if stop is not None and stop.is_set():
                return -1
        with self._load_lock:
            w = min(range(self.n), key=lambda i: self.load[i])
            self.load[w] += 1
        self.tqs[w].put(msg)
        return w

    def done(self, wid: int):
        with self._load_lock:
            self.load[wid] -= 1
        self.slots.release()

    def close(self, timeout: float = 60.0):
        for q in self.tqs:
            try:
                q.put(None)
            except Exception:  # noqa: BLE001
                pass
        t0 = time.time()
        for p in self.procs:
            p.join(max(0.1, timeout - (time.time() - t0)))
            if p.is_alive():
                p.terminate()
                p.join(5)


# ------------------------------------------------------------------------------------------
# the coordinator
# ------------------------------------------------------------------------------------------
@dataclasses.dataclass
class _FamilyIndex:
    """What the coordinator keeps of a sent batch: enough for pipeline.consensus_from_output."""

    fam_mi: np.ndarray
    fam_off: np.ndarray
    src: np.ndarray

    @property
    def n_fam(self) -> int:
        return int(self.fam_off.shape[0]) - 1


def step5_stream_multi(in_bam: str, fasta: str, out_bam: Optional[str], devices: Sequence[int],
                       prefix: Optional[str] = None, threads: int = 0, level: int = 6,
                       fastq: Optional[Tuple[str, str]] = None, tags: bool = True, chunk_bytes: Optional[int] = None,
                       slack: Optional[int] = None, batch_bases: Optional[int] = None, inflight: int = 2,
                       runner: Optional[str] = None, stats: Optional[dict] = None, gpu_bgzf: bool = False,
                       fleet: Optional["Fleet"] = None) -> dict:
    """bam.step5_stream over len(devices) GPU workers (see the module docstring).  Same file
    contract and output bytes as bam.step5 / bam.step5_stream (main.snake.py:121-164).
    gpu_bgzf: the writer deflates on devices[0] (bam.GpuBgzf; the coordinator touches that GPU
    only after its workers are spawned).  fleet: an already started Fleet over `devices` (left
    running; e.g. to time the stream without the workers' start-up), else one is started and
    closed here."""
    from . import bam, pipeline
    chunk_bytes = bam.DEFAULT_CHUNK_BYTES if chunk_bytes is None else chunk_bytes
    slack = bam.DEFAULT_SLACK if slack is None else slack
    T = {"decode": 0.0, "plan": 0.0, "materialize": 0.0, "submit_wait": 0.0, "records": 0.0, "encode": 0.0}
    info = {"records_in": 0, "families": 0, "families_emitted": 0, "records_out": 0, "chunks": 0, "batches": 0,
            "workers": len(devices)}
    hdr0 = bam.read_bam_header(in_bam)
    ref = bam.read_fasta(fasta, hdr0)
    pre = bam.read_name_prefix(hdr0) if prefix is None else prefix
    tg = tags and out_bam is not None  # the FASTQ pair carries no tags
    mode = pipeline.MODE_CONVERT | pipeline.MODE_EXTEND | pipeline.MODE_VOTE
    own_fleet = fleet is None
    fleet = Fleet(devices, runner, inflight) if own_fleet else fleet
    # batch images and messages; a batch's go back when its result arrives; a dropped one is
    # forgotten by every worker (fleet.broadcast is thread-safe: mp queues)
    cpool = SegmentPool("c", on_drop=lambda name: fleet.broadcast(("forget", name)))
    # the segments the in-flight batches need, faulted in while the first chunk is read: a batch's
    # images are about 0.75 x its record bytes (bounded by the batch base budget too)
    est = int(0.75 * chunk_bytes)
    if batch_bases:
        est = min(est, int(1.7 * batch_bases))
    nseg = fleet.slots_total + 3  # (+ the batches the planner has materialized ahead of the dealer)
    cpool.prefill(nseg, int(1.25 * est) + 4096)
    cpool.prefill(nseg, SegmentPool.MIN)
    views = SegmentViews()  # the workers' result segments
    stop = threading.Event()
    err: List[BaseException] = []
    raws: "queue.Queue" = queue.Queue(maxsize=1)
    parsed: "queue.Queue" = queue.Queue(maxsize=1)
    chunks: "queue.Queue" = queue.Queue(maxsize=1)
    outs: "queue.Queue" = queue.Queue(maxsize=1)
    # chunk id -> {"raw", "n" (batches; None until the dealer has sent them all), "parts": {i:
    # Consensus}, "index": {i: _FamilyIndex}, "in": {i: coordinator segments of batch i}, "out":
    # [(worker, its result segments)]}, filled by the dealer and the collector
    pend: Dict[int, dict] = {}
    eof: List[Optional[int]] = [None]  # number of chunks, once the dealer has seen them all
    plock = threading.Condition()

    def fail(e: BaseException):
        err.append(e)
        stop.set()
        with plock:
            plock.notify_all()

    bufs = bam.BufferPool()  # a chunk's record and tag arrays, given back once it is written
    R_: dict = {}  # the reader's steps (StreamChunk.decode timing)

    def decoder():  # cuts the next chunk while the planner decodes and plans the one before
        it = None
        try:
            it = bam.stream_chunks(in_bam, threads, chunk_bytes, slack)
            for ch in it:
                if stop.is_set():
                    ch.discard()
                    break
                raws.put(ch)
        except BaseException as e:  # noqa: BLE001
            fail(e)
        finally:
            if it is not None:
                it.close()
            raws.put(None)

    def reader():  # parses a chunk's records while the planner forms the families of the one before
        try:
            while True:
                t0 = time.perf_counter()
                ch = raws.get()
                if ch is None:
                    break
                if stop.is_set():
                    ch.discard()
                    continue  # drain to the decoder's None
                t1 = time.perf_counter()
                raw = ch.decode(threads, R_, bufs)[1]
                T["parse"] = T.get("parse", 0.0) + time.perf_counter() - t1
                T["decode"] += t1 - t0  # the wait for the decoder
                parsed.put(raw)
        except BaseException as e:  # noqa: BLE001
            fail(e)
            while True:
                ch = raws.get()
                if ch is None:
                    break
                ch.discard()
        finally:
            parsed.put(None)

    def materialize(plan, a: int, b: int):
        """-> (the batch without its host bookkeeping, its _FamilyIndex, the segments it uses)."""
        img = []

        def images(n_slots: int):  # the family images straight into a shared segment
            ns = (n_slots // 2 + 255) // 256 * 256
            img.append(cpool.take(ns + n_slots + 256))
            buf = np.frombuffer(cpool.buf(img[-1]), np.uint8)
            return buf[:ns], buf[ns:ns + n_slots]
        fb = pipeline.materialize(plan, a, b, images=images)
        index = _FamilyIndex(fb.fam_mi.copy(), fb.fam_off.astype(np.int64), fb.src.astype(np.int64))
        # the worker needs the device arrays only (host bookkeeping stays here)
        slim = dataclasses.replace(fb, src=np.zeros(0, np.int64), fam_mi=np.zeros(0, np.int32),
                                   t2_rank=np.zeros(0, np.int64), rec_tid=np.zeros(0, np.int32))
        return slim, index, img

    def planner():  # forms a chunk's families and materializes its batches ahead of the dealer
        try:
            while True:
                raw = parsed.get()
                if raw is None:
                    break
                if stop.is_set():
                    continue  # drain to the reader's None
                t0 = time.perf_counter()
                plan = pipeline.plan_families(raw, "full", ref)
                t1 = time.perf_counter()
                T["plan"] += t1 - t0
                batches = None if plan.split_ext else [materialize(plan, a, b)
                                                       for a, b in pipeline.plan_ranges(plan, batch_bases)]
                T["materialize"] += time.perf_counter() - t1
                chunks.put((raw, plan, batches))
        except BaseException as e:  # noqa: BLE001
            fail(e)
            while parsed.get() is not None:
                pass
        finally:
            chunks.put(None)

    def collector():
        """Worker results -> pend; complete chunks go to the writer in input order."""
        nxt = 0
        try:
            while not stop.is_set():
                ready = []
                with plock:
                    while nxt in pend and pend[nxt]["n"] is not None and len(pend[nxt]["parts"]) == pend[nxt]["n"]:
                        ready.append(pend.pop(nxt))
                        nxt += 1
                    if ready:
                        plock.notify_all()
                    finished = eof[0] is not None and nxt >= eof[0]
                for c in ready:
                    outs.put(c)
                if finished:
                    break
                m = fleet.get(timeout=0.5)
                if m is None:
                    continue
                if m[0] == "forget":  # a worker dropped one of its result segments
                    views.forget(m[2])
                    continue
                kind, wid, (cid, i), res = m[0], m[1], m[2], unpack(m[3], views)
                for k, v in m[5].items():  # (the workers' busy time, summed)
                    T[k] = T.get(k, 0.0) + v
                with plock:
                    c = pend[cid]
                    c["parts"][i] = pipeline.consensus_from_output(c["index"].pop(i), res) if kind == "batch" else res
                    c["out"].append((wid, m[4]))
                    back = c["in"].pop(i, ())
                    plock.notify_all()
                for name in back:  # (the worker has read the batch: its result is back)
                    cpool.give(name)
                fleet.done(wid)
        except BaseException as e:  # noqa: BLE001
            fail(e)
        finally:
            outs.put(None)

    def writer():
        w = fq = None
        try:
            gz = bam.GpuBgzf(int(devices[0])) if gpu_bgzf and out_bam is not None else None
            gzf = bam.GpuBgzf(int(devices[0])) if gpu_bgzf and fastq is not None else None
            w = bam.BamWriter(out_bam, bam.output_header(hdr0), level, gz) if out_bam is not None else None
            fq = bam.FastqWriter(fastq[0], fastq[1], level, gzf) if fastq is not None else None
            while True:
                c = outs.get()
                if c is None:
                    break
                if stop.is_set():
                    continue
                cons = pipeline.concat_consensus([c["parts"][i] for i in range(c["n"])])
                info["families"] += int(cons.status.shape[0])
                info["families_emitted"] += int(((cons.status & 1) != 0).sum())
                t0 = time.perf_counter()
                recs = bam.duplex_records(cons, c["raw"], pre, threads, pool=bufs)
                t1 = time.perf_counter()
                if w is not None:
                    w.add(recs, threads)
                if fq is not None:
                    fq.add(recs, threads)
                info["records_out"] += recs.n
                T["records"] += t1 - t0
                T["encode"] += time.perf_counter() - t1
                back = [getattr(c["raw"], "_pool_buf", None), getattr(recs.aux2, "_pool_buf", None)]
                results = c["out"]
                del c, cons, recs
                for buf in back:  # (the chunk is written: nothing refers to its record arrays)
                    bufs.give(buf)
                for wid, names in results:  # nor to the workers' result segments
                    for name in names:
                        fleet.tqs[wid].put(("release", name))
            if not stop.is_set():
                if w is not None:
                    w.close(threads)
                if fq is not None:
                    fq.close(threads)
            else:
                bam.close_quietly(w, fq)
        except BaseException as e:  # noqa: BLE001
            fail(e)
            bam.close_quietly(w, fq)
            while outs.get() is not None:
                pass

    workers = [threading.Thread(target=f, daemon=True) for f in (decoder, reader, planner, collector, writer)]
    drained = False
    try:
        fleet.broadcast(("ref", pack(dataclasses.replace(ref, letters={}), cpool)[0]))
        for t in workers:
            t.start()
        cid = 0
        while not stop.is_set():
            item = chunks.get()
            if item is None:
                drained = True
                break
            raw, plan, batches = item
            info["records_in"] += raw.n
            info["chunks"] += 1
            with plock:  # a bounded number of chunks between the dealer and the writer
                while len(pend) >= 2 * fleet.n + 2 and not stop.is_set():
                    plock.wait(0.5)
                pend[cid] = {"raw": raw, "n": None, "parts": {}, "index": {}, "in": {}, "out": []}
            n = 0
            if plan.split_ext:
                t, segs = pack(raw, cpool)
                with plock:
                    pend[cid]["in"][0] = segs
                if fleet.submit(("chunk", (cid, 0), t, tg, batch_bases), stop) >= 0:
                    n = 1
            else:
                for slim, index, img in batches:
                    raw_sub = R.take(raw, index.src) if fleet.needs_raw else None
                    t0 = time.perf_counter()
                    t, segs = pack(slim, cpool)
                    rt, rsegs = pack(raw_sub, cpool) if raw_sub is not None else (None, [])
                    T["pack"] = T.get("pack", 0.0) + time.perf_counter() - t0
                    with plock:
                        pend[cid]["index"][n] = index
                        pend[cid]["in"][n] = sorted(set(segs) | set(rsegs) | set(img))
                    t0 = time.perf_counter()
                    w = fleet.submit(("batch", (cid, n), t, mode, tg, rt), stop)
                    T["submit_wait"] += time.perf_counter() - t0
                    del slim, raw_sub
                    if w < 0:
                        break
                    n += 1
                    info["batches"] += 1
                del batches
            with plock:
                pend[cid]["n"] = n
                plock.notify_all()
            cid += 1
        with plock:
            eof[0] = cid
            plock.notify_all()
    except BaseException as e:  # noqa: BLE001
        fail(e)
    finally:
        if not drained:  # let the planner and the decoder finish (they stop at their next chunk)
            stop.set()
            while chunks.get() is not None:
                pass
        for t in workers:
            t.join(timeout=600)
        if own_fleet:
            fleet.close()
        else:  # (a kept fleet's workers may still hold this run's result segments: let them go)
            for wid in range(fleet.n):
                fleet.tqs[wid].put(("drop",))
        views.close()
        cpool.close()
    if err:
        raise err[0]
    if stats is not None:
        stats.update({k: round(v, 4) for k, v in T.items()})
        stats.update({"reader_" + k: round(v, 4) for k, v in R_.items()})
        stats["segments_created"] = cpool.n
        stats["segments_created_MiB"] = round(cpool.created_bytes / 2**20, 1)
    return info
