#!/bin/bash
# Round-4 session g6: reciprocal-free GELU (gelu_erf2x2) -- GEMM/encoder/transform
# parity tests, the A/B against the previous build on the GELU/GEGLU shapes, and
# the encoder bench under rocprof.
set -o pipefail
OUT=gpurun_out/${1:-r4g6}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu \
  tests/test_gemm_half_tail.py tests/test_gemm_chunked.py tests/test_lnfold.py tests/test_gpu_parity.py \
  tests/test_encoder.py tests/test_auc_gate.py > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc" > "$OUT/status.txt"; [ $rc -eq 0 ] || exit $rc
L=news_recommendation_project_v2_amd/libnewsrec_hip.so
timeout -k 10 300 python -u tools/gemm_ab.py --libs new=$L old=tools/gemm_lab/libnewsrec_oldgelu.so --rounds 5 \
  --shapes probe,latent.ff1,latent.S > "$OUT/gemm_ab.jsonl" 2> "$OUT/gemm_ab.err"
echo "gemm_ab rc=$?" >> "$OUT/status.txt"
timeout -k 10 300 python -u tools/encoder_bench.py --n-news 16384 --dtype bf16 --reps 3 > "$OUT/encoder.json" 2> "$OUT/encoder.err"
echo "encoder rc=$?" >> "$OUT/status.txt"
