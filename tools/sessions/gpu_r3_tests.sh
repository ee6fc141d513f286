#!/bin/bash
# Round-3 GPU session 2: module-level training tests, the whole -m gpu suite, an N = 2 gloo
# rehearsal of bench.py's multi-rank path (ranks share the one GPU), then the default bench.
set -o pipefail
OUT=gpurun_out/${1:-r3b}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_final_attention_autograd.py > "$OUT/pytest_autograd.log" 2>&1 && \
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
  > "$OUT/pytest_gpu.log" 2>&1 && \
timeout -k 10 600 python -u bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 --cpu-seconds 0 \
  > "$OUT/bench_gloo2.json" 2> "$OUT/bench_gloo2.err" && \
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
