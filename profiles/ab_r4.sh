#!/bin/bash
# Round-4 A/B on the GPU box: bench per variant and config, no tests (run them first).  A variant is
# name=lib.so[:VAR=VALUE[,VAR=VALUE...]] ("-" for the in-tree library).
# Usage (repo root): CFGS="C2 C3 C4" bash profiles/ab_r4.sh <tag> <variant>...
set -u -o pipefail
TAG=$1; shift
OUT="$(pwd)/gpurun_out/$TAG"
mkdir -p "$OUT"
for c in ${CFGS:-C2 C3 C4}; do
  for v in "$@"; do
    name=${v%%=*}; rest=${v#*=}
    lib=${rest%%:*}; envs=""
    [ "$rest" != "$lib" ] && envs=${rest#*:}
    [ "$lib" = "-" ] && lib=bsseqconsensusreads_amd/libbsdc.so
    log="$OUT/bench_${c}_$name.log"
    env BSDC_LIB_PATH="$(realpath "$lib")" $(echo "$envs" | tr ',' ' ') \
      timeout -k 10 300 python -u bench.py --config "$c" --cpu-sample 0 --steps 20 > "$log" 2>&1 \
      || { echo "bench $c $name failed"; tail -20 "$log"; exit 1; }
    echo "$c $name $(tail -1 "$log" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r.get("small_kernel_ms"), r.get("large_kernel_ms"), d.get("tags_ms_per_step"))')"
  done
done
