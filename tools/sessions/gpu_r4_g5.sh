#!/bin/bash
# Round-4 session g5: epilogue cost at the ff1 shape (GEGLU vs none vs GELU), and a
# rocprof kernel trace of the bf16 title encoder (per-kernel split, round 4).
set -o pipefail
OUT=gpurun_out/${1:-r4g5}
mkdir -p "$OUT"
L=news_recommendation_project_v2_amd/libnewsrec_hip.so
timeout -k 10 300 python -u tools/gemm_ab.py --libs new=$L --rounds 5 --shapes probe,latent.ff1 \
  > "$OUT/gemm_ab.jsonl" 2> "$OUT/gemm_ab.err"
echo "gemm_ab rc=$?" > "$OUT/status.txt"
( cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_enc" -o enc --output-format csv -- \
  python tools/encoder_bench.py --n-news 16384 --dtype bf16 --reps 2 > "$OUT/encoder.json" 2> "$OUT/encoder.err" )
echo "encoder prof rc=$?" >> "$OUT/status.txt"
