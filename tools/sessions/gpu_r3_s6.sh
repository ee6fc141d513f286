#!/bin/bash
# Round-3 s6: encoder GPU tests (attention with an upper-bound launch), then rocprofv3
# kernel-traces of the bf16 title encoder at mean title length 20 and 66 tokens
# (the XCD-contiguous attention dispatch matters once a title spans several query blocks).
set -o pipefail
OUT=gpurun_out/${1:-r3s6}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_encoder.py \
  > "$OUT/pytest_encoder.log" 2>&1 && \
( cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/enc20" -o enc --output-format csv -- \
  python tools/encoder_bench.py --n-news 16384 --dtype bf16 > "$OUT/encoder_bench_len20.json" 2> "$OUT/encoder_bench_len20.err" ) && \
( cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/enc66" -o enc --output-format csv -- \
  python tools/encoder_bench.py --n-news 16384 --mean-len 66 --dtype bf16 > "$OUT/encoder_bench_len66.json" 2> "$OUT/encoder_bench_len66.err" )
