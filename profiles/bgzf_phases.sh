#!/bin/bash
# Builds libbsdc with the BGZF kernel's phase clocks (-DBSDC_BGZF_PHASES) into profiles/_build and
# runs profiles/bgzf_phases.py against it.  Usage: bash profiles/bgzf_phases.sh [out.log]
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
mkdir -p "$ROOT/profiles/_build"
if [ ! -f "$ROOT/profiles/_build/libbsdc_phases.so" ]; then
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared -DBSDC_BGZF_PHASES \
    -o "$ROOT/profiles/_build/libbsdc_phases.so" "$ROOT/bsseqconsensusreads_amd/csrc/bsdc_kernels.hip" \
    "$ROOT/bsseqconsensusreads_amd/csrc/bsdc_bgzf.hip"
fi
BSDC_LIB_PATH="$ROOT/profiles/_build/libbsdc_phases.so" timeout -k 10 200 python -u "$ROOT/profiles/bgzf_phases.py"
