"""ctypes binding of libbsdc (include/bsdc.h).  Loading fails loudly: there is no CPU fallback."""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# BSDC_LIB_PATH: an alternative build of the same library (profiling A/B runs only)
LIB_PATH = os.environ.get("BSDC_LIB_PATH") or os.path.join(HERE, "libbsdc.so")

BSDC_ABI_VERSION = 15
SMALL_BUCKETS = 8  # BSDC_SMALL_BUCKETS
LARGE_BUCKETS = 6  # BSDC_LARGE_BUCKETS
MODE_CONVERT, MODE_EXTEND, MODE_VOTE, MODE_DUMP = 1, 2, 4, 8
MODE_SKIP_SMALL, MODE_SKIP_LARGE = 16, 32
MODE_TAGS = 64  # single-strand reads + column statistics for the consensus tags


class Params(C.Structure):
    _fields_ = [("error_rate_pre_umi", C.c_double), ("error_rate_post_umi", C.c_double),
                ("min_input_base_quality", C.c_int32), ("consensus_call_overlapping_bases", C.c_int32),
                ("min_reads", C.c_int32), ("min_consensus_base_quality", C.c_int32)]


class FamilyBatchC(C.Structure):
    _fields_ = [("n_rec", C.c_int64), ("n_fam", C.c_int64),
                ("fam_off", C.c_void_p), ("rec", C.c_void_p), ("rec_win", C.c_void_p),
                ("cig_off", C.c_void_p), ("cig_info", C.c_void_p), ("cigar", C.c_void_p),
                ("rt", C.c_void_p), ("seq", C.c_void_p), ("qual", C.c_void_p),
                ("small_fams", C.c_void_p), ("n_small", C.c_int64 * SMALL_BUCKETS), ("small_arena", C.c_int32 * SMALL_BUCKETS),
                ("large_fams", C.c_void_p), ("n_large", C.c_int64 * LARGE_BUCKETS), ("large_arena", C.c_int32 * LARGE_BUCKETS),
                ("max_len", C.c_int32), ("split_part_arena", C.c_int32),
                ("split_parts", C.c_void_p), ("n_split_parts", C.c_int64), ("split_part_recs", C.c_void_p),
                ("split_fams", C.c_void_p),
                ("n_split_fams", C.c_int64), ("split_partial_off", C.c_int64)]


class ConsensusC(C.Structure):
    _fields_ = [("stride", C.c_int32), ("reserved", C.c_int32),
                ("status", C.c_void_p), ("len", C.c_void_p), ("seq", C.c_void_p), ("qual", C.c_void_p),
                ("dump_pos", C.c_void_p), ("dump_len", C.c_void_p), ("dump_tags", C.c_void_p),
                ("dump_seq", C.c_void_p), ("dump_qual", C.c_void_p), ("scratch", C.c_void_p),
                ("ss_len", C.c_void_p), ("ss_base", C.c_void_p), ("ss_qual", C.c_void_p), ("ss_depth", C.c_void_p),
                ("ss_err", C.c_void_p), ("ss_wide", C.c_void_p), ("ss_wdepth", C.c_void_p), ("ss_werr", C.c_void_p)]


EXPORTS = ("bsdc_abi_version", "bsdc_ctx_create", "bsdc_ctx_set_params", "bsdc_ctx_destroy", "bsdc_last_error",
           "bsdc_load_reference", "bsdc_run", "bsdc_convert", "bsdc_extend", "bsdc_duplex_call",
           "bsdc_family_arena_bytes", "bsdc_small_arena_bytes", "bsdc_get_tables", "bsdc_model_tables",
           "bsdc_model_tables_fp64", "bsdc_agree_tables", "bsdc_phred_buckets", "bsdc_bgzf_scratch_bytes",
           "bsdc_bgzf_deflate", "bsdc_bgzf_pack", "bsdc_host_register", "bsdc_host_unregister")

_lib = None


def load(path: str = LIB_PATH):
    """Load libbsdc.so (built by __graft_entry__.build()); raises if it is missing."""
    global _lib
    if _lib is not None and path == LIB_PATH:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError("libbsdc.so not built (%s): run `python -c 'import __graft_entry__ as g; g.build()'`" % path)
    lib = C.CDLL(path)
    lib.bsdc_abi_version.restype = C.c_int32
    lib.bsdc_ctx_create.argtypes = [C.c_int32, C.POINTER(Params), C.POINTER(C.c_void_p)]
    lib.bsdc_ctx_create.restype = C.c_int32
    lib.bsdc_ctx_set_params.argtypes = [C.c_void_p, C.POINTER(Params)]
    lib.bsdc_ctx_set_params.restype = C.c_int32
    lib.bsdc_ctx_destroy.argtypes = [C.c_void_p]
    lib.bsdc_ctx_destroy.restype = None
    lib.bsdc_last_error.argtypes = [C.c_void_p]
    lib.bsdc_last_error.restype = C.c_char_p
    lib.bsdc_load_reference.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_int32]
    lib.bsdc_load_reference.restype = C.c_int32
    lib.bsdc_run.argtypes = [C.c_void_p, C.POINTER(FamilyBatchC), C.POINTER(ConsensusC), C.c_int32, C.c_void_p]
    lib.bsdc_run.restype = C.c_int32
    for fn in ("bsdc_convert", "bsdc_extend"):
        getattr(lib, fn).argtypes = [C.c_void_p, C.POINTER(FamilyBatchC), C.POINTER(ConsensusC), C.c_void_p]
        getattr(lib, fn).restype = C.c_int32
    lib.bsdc_duplex_call.argtypes = [C.c_void_p, C.POINTER(FamilyBatchC), C.POINTER(ConsensusC), C.c_int32, C.c_void_p]
    lib.bsdc_duplex_call.restype = C.c_int32
    lib.bsdc_family_arena_bytes.argtypes = [C.c_int32, C.c_int64, C.c_int32, C.c_int64]
    lib.bsdc_family_arena_bytes.restype = C.c_int64
    lib.bsdc_small_arena_bytes.argtypes = [C.c_int32, C.c_int64, C.c_int32, C.c_int64, C.c_int32]
    lib.bsdc_small_arena_bytes.restype = C.c_int64
    lib.bsdc_get_tables.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    lib.bsdc_get_tables.restype = C.c_int32
    lib.bsdc_model_tables.argtypes = [C.c_double, C.c_double, C.c_void_p, C.c_void_p]
    lib.bsdc_model_tables.restype = None
    lib.bsdc_model_tables_fp64.argtypes = [C.c_double, C.c_double, C.c_void_p, C.c_void_p]
    lib.bsdc_model_tables_fp64.restype = None
    lib.bsdc_agree_tables.argtypes = [C.c_double, C.c_double, C.c_void_p, C.c_void_p]
    lib.bsdc_agree_tables.restype = None
    lib.bsdc_bgzf_scratch_bytes.argtypes = [C.c_int64]
    lib.bsdc_bgzf_scratch_bytes.restype = C.c_int64
    lib.bsdc_bgzf_deflate.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p]
    lib.bsdc_bgzf_deflate.restype = C.c_int32
    lib.bsdc_bgzf_pack.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int64, C.c_void_p, C.c_void_p]
    lib.bsdc_bgzf_pack.restype = C.c_int32
    lib.bsdc_host_register.argtypes = [C.c_int32, C.c_void_p, C.c_int64]
    lib.bsdc_host_register.restype = C.c_int32
    lib.bsdc_host_unregister.argtypes = [C.c_int32, C.c_void_p]
    lib.bsdc_host_unregister.restype = C.c_int32
    lib.bsdc_phred_buckets.argtypes = [C.c_double, C.c_double, C.c_void_p]
    lib.bsdc_phred_buckets.restype = None
    if lib.bsdc_abi_version() != BSDC_ABI_VERSION:
        raise RuntimeError("libbsdc ABI %d != %d" % (lib.bsdc_abi_version(), BSDC_ABI_VERSION))
    if path == LIB_PATH:
        _lib = lib
    return lib
