#!/bin/bash
# Round-3 s4: GEMM A/B of the shipped persistent kernel vs hipBLASLt on the 8 transform shapes,
# then a rocprofv3 kernel-trace of the bf16 title encoder (per-kernel breakdown).
set -o pipefail
OUT=gpurun_out/${1:-r3ge}
mkdir -p "$OUT"
timeout -k 10 300 python -u tools/gemm_ab.py --rounds 5 --libs new=news_recommendation_project_v2_amd/libnewsrec_hip.so > "$OUT/gemm_ab.jsonl" 2> "$OUT/gemm_ab.err" && \
( cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/enc_trace" -o enc --output-format csv -- \
  python tools/encoder_bench.py --n-news 16384 --dtype bf16 > "$OUT/encoder_bench.json" 2> "$OUT/encoder_bench.err" )
