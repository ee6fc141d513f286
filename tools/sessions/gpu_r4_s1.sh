#!/bin/bash
# Round-4 session 1: new GPU tests first (comm, residency flush, bf16 drift vs the
# oracle, AUC gate with logistic labels), then the whole -m gpu suite, smoke, the
# default bench, and the 2-rank gloo bench (multi-rank plumbing + dist info).
set -o pipefail
OUT=gpurun_out/${1:-r4s1}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu -s \
  tests/test_comm.py tests/test_residency.py tests/test_train_bf16_drift.py > "$OUT/pytest_new.log" 2>&1 && \
timeout -k 10 1000 python -u -m pytest -v --timeout 600 --timeout-method thread -m gpu -s \
  --deselect tests/test_train_bf16_drift.py --deselect tests/test_comm.py tests/ > "$OUT/pytest_gpu.log" 2>&1
rc=$?
echo "pytest rc=$rc" > "$OUT/status.txt"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 && \
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" && \
timeout -k 10 400 python -u bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 --cpu-seconds 0 \
  > "$OUT/bench_gloo2.json" 2> "$OUT/bench_gloo2.err"
echo "tail rc=$?" >> "$OUT/status.txt"
