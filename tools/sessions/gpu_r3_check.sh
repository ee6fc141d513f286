#!/bin/bash
# Round-3 GPU session: new tests, the whole -m gpu suite, then the default bench.
set -o pipefail
OUT=gpurun_out/${1:-r3a}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_residency.py \
  tests/test_auc_gate.py tests/test_eval_multirank.py > "$OUT/pytest_new.log" 2>&1 && \
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
  > "$OUT/pytest_gpu.log" 2>&1 && \
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
