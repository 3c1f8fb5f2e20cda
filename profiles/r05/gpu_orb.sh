#!/bin/bash
# C4: parts keep a u8 OR per column instead of u8x4 counts without TAGS, and store a lane's 4
# columns as one dword + one 16-B vector.  Parity (both join arms), full-size C4, A/B vs HEAD,
# FETCH/WRITE per kernel instance.
set -u -o pipefail
TAG=$1
OUT="$(pwd)/gpurun_out/$TAG"
mkdir -p "$OUT"
B="$(pwd)/profiles/_build"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fp64.py -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
  || { echo "gpu tests failed"; grep -E "PASS|FAIL|Error|error" "$OUT/pytest.log" | tail -30; exit 1; }
tail -1 "$OUT/pytest.log"
# the opt-in fused-join arm, HEAD's library and this one (reported, not fatal)
for v in head new; do
  case $v in head) LP="$B/libbsdc_head.so";; *) LP="";; esac
  BSDC_LIB_PATH="$LP" BSDC_SPLIT_JOIN=part timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k split -q --timeout 300 --timeout-method thread > "$OUT/pytest_partjoin_$v.log" 2>&1
  echo "part-join $v rc=$?"; grep -E "^FAILED|passed|failed" "$OUT/pytest_partjoin_$v.log" | tail -8
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py -k "c4" -x -q --timeout 380 --timeout-method thread > "$OUT/pytest_c4.log" 2>&1 \
  || { echo "c4 tests failed"; grep -E "PASS|FAIL|Error|error" "$OUT/pytest_c4.log" | tail -30; exit 1; }
tail -1 "$OUT/pytest_c4.log"
for c in C4; do
  for v in head new head2 new2; do
    case $v in head*) LP="$B/libbsdc_head.so";; *) LP="";; esac
    BSDC_LIB_PATH="$LP" timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 2 --cpu-sample 0 > "$OUT/bench_${c}_$v.log" 2>&1 || { tail -20 "$OUT/bench_${c}_$v.log"; exit 1; }
    tail -1 "$OUT/bench_${c}_$v.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$c $v ms', d['ms_per_step'], 'large_ms', r.get('large_kernel_ms'), 'tags_ms', d.get('tags_ms_per_step'))"
  done
done
R=$(pwd)
for v in head new; do
  case $v in head) LP="$B/libbsdc_head.so";; *) LP="";; esac
  i=0
  for grp in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    (cd /tmp && export TMPDIR=/tmp && BSDC_LIB_PATH="$LP" timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-include-regex 'k_small|k_large|k_join|k_tie' --output-format csv \
      -d "$OUT/pmc_$v/p$i" -o pmc -- python3 "$R/bench.py" --config C4 --steps 3 --warmup 1 --cpu-sample 0 --no-tags-leg > "$OUT/pmc_${v}_$i.log" 2>&1) || { echo "pmc $v $i failed"; tail -5 "$OUT/pmc_${v}_$i.log"; exit 1; }
  done
  python3 - "$OUT/pmc_$v" <<'PY'
import csv, glob, sys, collections
per = collections.defaultdict(float)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0] + " wg=" + r["Workgroup_Size"]
        per[(k, r["Counter_Name"], f, int(r["Dispatch_Id"]))] += float(r["Counter_Value"])
agg = collections.defaultdict(list)
for (k, c, f, d), v in per.items(): agg[(k, c)].append(v)
tot = 0.0
for (k, c), v in sorted(agg.items()):
    m = sum(v) / len(v) * 1024 * (2 if c == "FETCH_SIZE" else 1)  # (coalesced reads: FETCH_SIZE is half, profiles/calib_fetch.sh)
    if not k.startswith("k_small"): tot += m * len(v) / 4  # per step: 4 steps (1 warmup + 3) under the profiler
    print("%s %-45s %-10s n=%3d  %8.1f MB per dispatch" % (sys.argv[1].split("_")[-1], k[:45], c, len(v), m / 1e6))
print("large set HBM bytes per step: %.3f GB" % (tot / 1e9))
PY
done
