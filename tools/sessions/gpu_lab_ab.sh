#!/bin/bash
# GEMM lab A/B: the shipped library against the lab builds named in $LABS (name=path ...),
# the 8 transform shapes (tools/gemm_ab.py) and both whole transforms (tools/transform_ab.py).
set -o pipefail
OUT=gpurun_out/${1:-lab}
mkdir -p "$OUT"
timeout -k 10 300 python -u tools/gemm_ab.py --rounds 5 --libs new=news_recommendation_project_v2_amd/libnewsrec_hip.so $LABS \
  > "$OUT/gemm_ab.jsonl" 2> "$OUT/gemm_ab.err" && \
timeout -k 10 300 python -u tools/transform_ab.py --libs new=news_recommendation_project_v2_amd/libnewsrec_hip.so $LABS \
  > "$OUT/transform_ab.jsonl" 2> "$OUT/transform_ab.err"
