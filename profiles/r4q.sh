#!/bin/bash
# Round-4: where step 1's upload time goes (profiles/upload_probe.py), then step 1's stream end to
# end with the vectorised run names, and its GPU tests.
set -u -o pipefail
OUT=gpurun_out/r4q
mkdir -p $OUT
timeout -k 10 300 python -u profiles/upload_probe.py > $OUT/upload_probe.log 2>&1 || { tail -20 $OUT/upload_probe.log; exit 1; }
cat $OUT/upload_probe.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_parity.py -m gpu -x -q -k "molecular" --timeout 300 \
  --timeout-method thread > $OUT/pytest_mol.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $OUT/pytest_mol.log | head; exit 1; }
tail -1 $OUT/pytest_mol.log
timeout -k 10 600 python -u profiles/e2e_stream.py --families 1000000 --threads 16 --modes molecular_stream > $OUT/e2e.log 2>&1 || { tail -20 $OUT/e2e.log; exit 1; }
grep -E "^molecular_stream" $OUT/e2e.log | cut -c1-900
