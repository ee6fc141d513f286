#!/bin/bash
# Round-4 session g8: encoder LayerNorm folding -- its tests + the encoder and GEMM
# tests, then the interleaved fold on / off encoder A/B.
set -o pipefail
OUT=gpurun_out/${1:-r4g8}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
  tests/test_encoder_lnfold.py tests/test_encoder.py tests/test_gemm_half_tail.py tests/test_lnfold.py \
  > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc" > "$OUT/status.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/encoder_bench.py --n-news 16384 --dtype bf16 --reps 3 --ab-ln-fold \
  > "$OUT/encoder_ab.json" 2> "$OUT/encoder_ab.err"
echo "encoder ab rc=$?" >> "$OUT/status.txt"
