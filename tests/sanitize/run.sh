#!/bin/bash
# Host sanitizer run ("ASan/UBSan on host C++"): the host codec libbsdc_io
# (BGZF/BAM parsing of untrusted bytes, include/bsdc_io.h) and the oracle/ restatement rebuilt
# with -fsanitize=address,undefined, then the CPU tests that drive them -- round trips, corrupt,
# truncated and malformed BAMs (tests/test_bam.py), family formation (tests/test_families.py, and
# the C++ family formation bsdc_host.cpp against its numpy statement, tests/test_host_plan.py),
# the golden fixtures (tests/test_oracle_golden.py), the BGZF restatement and the writer's
# GPU-compressed path with its CPU stand-in (tests/test_bgzf.py), the stream with deferred far templates
# (tests/test_long_span.py) and the rank processes (tests/test_ranks.py) -- loaded against the instrumented builds.
# CPU only (GPU sanitizers are not available on the MI355X pool).  Usage: tests/sanitize/run.sh
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/../.." && pwd)"
OUT="$ROOT/build/sanitize"
mkdir -p "$OUT"
SAN="-fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer -g -O1"
g++ -std=c++17 -fopenmp -fPIC -shared -Wall $SAN -o "$OUT/libbsdc_io.so" \
    "$ROOT/bsseqconsensusreads_amd/csrc/bsdc_io.cpp" "$ROOT/bsseqconsensusreads_amd/csrc/bsdc_host.cpp" -lz -ldl
gcc -fopenmp -fPIC -shared -ffp-contract=off -Wall $SAN -o "$OUT/liboracle.so" "$ROOT/oracle/bsdc_oracle.c" "$ROOT/oracle/bgzf_ref.c" -lm
# python itself is not instrumented: the runtimes go in first; leak checking is off (the
# interpreter keeps its arenas to exit)
export LD_PRELOAD="$(gcc -print-file-name=libasan.so) $(gcc -print-file-name=libubsan.so)"
export ASAN_OPTIONS="detect_leaks=0:verify_asan_link_order=0:abort_on_error=1:halt_on_error=1"
export UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1"
export BSDC_IO_LIB_PATH="$OUT/libbsdc_io.so" BSDC_ORACLE_LIB="$OUT/liboracle.so"
cd "$ROOT"
# the instrumented builds are the ones loaded
python -c "
from bsseqconsensusreads_amd import bam
from oracle import oracle
bam._load(); oracle.load()
maps = open('/proc/self/maps').read()
assert '$OUT/libbsdc_io.so' in maps and '$OUT/liboracle.so' in maps, 'instrumented libraries not loaded'
print('sanitizer builds loaded:', '$OUT')
"
python -m pytest -q -p no:cacheprovider tests/test_bam.py tests/test_families.py tests/test_oracle_golden.py \
    tests/test_host_plan.py tests/test_bgzf.py tests/test_stream.py tests/test_long_span.py tests/test_ranks.py "$@"
