#!/bin/bash
# Round-4 GEMM session 1: the half-tile tail -- its bit-identity tests, the
# per-shape A/B against itself (tail off) and hipBLASLt, the whole transform A/B.
set -o pipefail
OUT=gpurun_out/${1:-r4g1}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gemm_half_tail.py tests/test_gemm_chunked.py > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc" > "$OUT/status.txt"; [ $rc -eq 0 ] || exit $rc
L=news_recommendation_project_v2_amd/libnewsrec_hip.so
timeout -k 10 300 python -u tools/gemm_ab.py --libs tail=$L notail=$L:notail --rounds 5 \
  --shapes final.l1,final.l3,final.l5,latent > "$OUT/gemm_ab.jsonl" 2> "$OUT/gemm_ab.err"
rc=$?; echo "gemm_ab rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/half_tail_ab.py > "$OUT/transform_ab.jsonl" 2> "$OUT/transform_ab.err"
echo "transform_ab rc=$?" >> "$OUT/status.txt"
