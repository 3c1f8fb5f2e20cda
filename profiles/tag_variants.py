"""Tag-leg ablation (profiling only, never shipped): builds variants of
libbsdc.so whose TAGS instance of k_small drops one piece of the tag work each, into
profiles/_build/libbsdc_<name>.so, so that bench.py's tags leg (BSDC_LIB_PATH=...) prices each piece.
Their tag outputs are wrong by construction; the untagged instance is untouched.
  nofast:  no single-strand stores (nor read counts) in the vote's fast path
  noqueue: no single-strand stores (nor per-base counts) in the queued columns' path
  ollen:   the vote loop runs to the duplex length, not the single strands' longer one
  bare:    all three
  st1/st2/st3: the fast path's full-dword stores cut to ss_base / + ss_qual / + ss_depth
  nocount: no per-column read counts in the fast path (depth stored as 0)
(the st* variants edit the whole-dword stores of round 6; round 6's first ablation ran them on
the byte-masked stores before it)
Usage (CPU, this container): python profiles/tag_variants.py"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "bsseqconsensusreads_amd", "csrc")
OUT = os.path.join(ROOT, "profiles", "_build")

FAST = ("if (TAGS && c < lv) {", "if (false && TAGS && c < lv) {")
QUEUE = ("if (TAGS) {  // this side's single-strand column", "if (false) {  // this side's single-strand column")
OLLEN = ("const int lv = TAGS ? ::max(la, lb) : ol;", "const int lv = ol;")
ST_Q = ("                        *reinterpret_cast<uint32_t *>(P.O.ss_qual + at) = ss[2 * side + 1];\n", "")
ST_D = ("                        *reinterpret_cast<uint32_t *>(P.O.ss_depth + at) = n4;\n", "")
ST_E = ("                        *reinterpret_cast<uint32_t *>(P.O.ss_err + at) = 0u;\n", "")
NOCOUNT = ("const uint32_t n4 = nf[side] + __builtin_bswap32(nr[side]);", "const uint32_t n4 = 0u;")
VARIANTS = {"nofast": [FAST], "noqueue": [QUEUE], "ollen": [OLLEN], "bare": [FAST, QUEUE, OLLEN],
            "st1": [ST_Q, ST_D, ST_E], "st2": [ST_D, ST_E], "st3": [ST_E], "nocount": [NOCOUNT]}


def main():
    src = open(os.path.join(CSRC, "bsdc_kernels.hip")).read()
    os.makedirs(OUT, exist_ok=True)
    only = sys.argv[1:]
    for name, edits in VARIANTS.items():
        if only and name not in only:
            continue
        s = src
        for a, b in edits:
            assert s.count(a) == 1, (name, a)
            s = s.replace(a, b)
        tmp = os.path.join(CSRC, "_var_%s.hip" % name)
        with open(tmp, "w") as fh:
            fh.write(s)
        try:
            cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC",
                   "-shared", "-w", "-o", os.path.join(OUT, "libbsdc_%s.so" % name), tmp,
                   os.path.join(CSRC, "bsdc_bgzf.hip")]
            print(name, flush=True)
            subprocess.run(cmd, check=True)
        finally:
            os.unlink(tmp)


if __name__ == "__main__":
    sys.exit(main())
