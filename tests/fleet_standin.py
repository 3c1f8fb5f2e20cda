"""A CPU stand-in for fleet.GpuRunner (TEST INFRASTRUCTURE ONLY): computes a batch's output arrays
with oracle/ instead of the kernels, in the exact layout DeviceBatch.fetch returns, so that the
multi-process streaming path (bsseqconsensusreads_amd/fleet.py: spawn, chunks, shared-memory
hand-off, ordering, writer) runs on a machine without a GPU (tests/test_fleet.py).

It asks for each batch's records (needs_raw): the families of a batch are complete and
contiguous in TemplateCoordinate order, so oracle/ on those records alone forms the same families
in the same order, which run_batch checks before answering."""
from __future__ import annotations

import numpy as np

from bsseqconsensusreads_amd.batch import round16, wide_rows
from oracle import oracle


def _pack_rows(codes: np.ndarray) -> np.ndarray:
    """[..., stride] nt16 codes -> [..., stride / 2] bytes, high nibble first (BAM order)."""
    return ((codes[..., 0::2] << 4) | codes[..., 1::2]).astype(np.uint8)


class OracleRunner:
    needs_raw = True

    def __init__(self, device: int):
        self.ref = None

    def load_reference(self, ref):
        self.ref = ref

    def _result(self, raw):
        return oracle.run(raw, self.ref, threads=2)

    def run_batch(self, fb, mode: int, tags: bool, raw_sub=None) -> dict:
        r = self._result(raw_sub)
        F = fb.n_fam
        # the batch's families, as oracle/ forms them on its records: same sizes, same order
        assert np.array_equal(np.diff(r.fam_rec_off), np.diff(fb.fam_off.astype(np.int64))), "family sizes"
        assert np.array_equal(r.fam_src, np.arange(raw_sub.n)), "family order"
        stride = int(round16(max(int(fb.max_len) + 2, r.cons_seq.shape[2])))

        def pad(a):
            return np.pad(a, [(0, 0)] * (a.ndim - 1) + [(0, stride - a.shape[-1])])
        ss_len = r.ss["len"].astype(np.int32)
        status = (r.status & 1).astype(np.uint8)
        status |= np.where((ss_len[:, 0] > 0) | (ss_len[:, 1] > 0), 2, 0).astype(np.uint8)
        status |= np.where((ss_len[:, 2] > 0) | (ss_len[:, 3] > 0), 4, 0).astype(np.uint8)
        live = np.arange(stride)[None, None, :] < r.cons_len[:, :, None]
        out = {"status": status, "len": r.cons_len.astype(np.int32).reshape(F, 2),
               "seq": _pack_rows(np.where(live, pad(r.cons_seq), 0)), "qual": np.where(live, pad(r.cons_qual), 0),
               "stride": stride}
        if tags:
            live4 = np.arange(stride)[None, None, :] < ss_len[:, :, None]
            out.update(ss_len=ss_len, ss_base=np.where(live4, pad(r.ss["base"]), 0).astype(np.uint8),
                       ss_qual=np.where(live4, pad(r.ss["qual"]), 0).astype(np.uint8),
                       ss_depth=np.minimum(np.where(live4, pad(r.ss["depth"]), 0), 255).astype(np.uint8),
                       ss_err=np.minimum(np.where(live4, pad(r.ss["err"]), 0), 255).astype(np.uint8))
            wide, W = wide_rows(fb.fam_off)  # (the kernels' wide rows: families of 256+ records)
            f = np.nonzero(wide >= 0)[0]
            out.update(ss_wide=wide,
                       ss_wdepth=np.where(live4[f], pad(r.ss["depth"])[f], 0).astype(np.uint16),
                       ss_werr=np.where(live4[f], pad(r.ss["err"])[f], 0).astype(np.uint16))
        return out

    def run_chunk(self, raw, tags: bool, batch_bases):
        """A chunk whose tool-2 groups straddle its families (the streaming step's two-launch
        case): oracle/ on the whole chunk, as pipeline.run_step5's Consensus."""
        from bsseqconsensusreads_amd.pipeline import Consensus
        r = self._result(raw)
        F = int(r.status.shape[0])
        status = (r.status & 1).astype(np.uint8)
        ss = None
        if tags:
            ss_len = r.ss["len"].astype(np.int32)
            status |= np.where((ss_len[:, 0] > 0) | (ss_len[:, 1] > 0), 2, 0).astype(np.uint8)
            status |= np.where((ss_len[:, 2] > 0) | (ss_len[:, 3] > 0), 4, 0).astype(np.uint8)
            ss = {"len": ss_len, "base": r.ss["base"], "qual": r.ss["qual"], "depth": r.ss["depth"], "err": r.ss["err"]}
        return Consensus(np.asarray(r.fam_mi, np.int32), status, r.cons_len.astype(np.int32).reshape(F, 2),
                         r.cons_seq, r.cons_qual, np.asarray(r.fam_rec_off, np.int64), np.asarray(r.fam_src, np.int64),
                         ss)

    def close(self):
        pass


class FailingRunner(OracleRunner):
    """Fails on its third batch (a worker dying mid-stream)."""

    def __init__(self, device: int):
        super().__init__(device)
        self.n = 0

    def run_batch(self, fb, mode: int, tags: bool, raw_sub=None) -> dict:
        self.n += 1
        if self.n == 3:
            raise ValueError("stand-in failure on batch 3")
        return super().run_batch(fb, mode, tags, raw_sub)
