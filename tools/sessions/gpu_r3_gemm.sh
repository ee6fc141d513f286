#!/bin/bash
# GEMM lab A/B: shipped persistent kernel (16x16x32) vs the MF32 variant (32x32x16), one process each tool.
set -o pipefail
OUT=gpurun_out/${1:-r3g1}
mkdir -p "$OUT"
L=tools/gemm_lab
timeout -k 10 600 python -u tools/gemm_ab.py --rounds 5 --libs new=news_recommendation_project_v2_amd/libnewsrec_hip.so \
  w4=$L/libnewsrec_w4.so > "$OUT/gemm_ab.jsonl" 2> "$OUT/gemm_ab.err" && \
timeout -k 10 300 python -u tools/transform_ab.py --libs new=news_recommendation_project_v2_amd/libnewsrec_hip.so \
  w4=$L/libnewsrec_w4.so > "$OUT/transform_ab.jsonl" 2> "$OUT/transform_ab.err"
