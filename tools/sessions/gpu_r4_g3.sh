#!/bin/bash
# Round-4 GEMM session 3: spill-free balanced-read kernel (rb3) -- GEMM + transform
# + training parity tests, then the per-shape A/B against rb2 and the round-start base.
set -o pipefail
OUT=gpurun_out/${1:-r4g3}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gemm_half_tail.py tests/test_gemm_chunked.py tests/test_lnfold.py tests/test_gpu_parity.py \
  tests/test_latent_attention_autograd.py tests/test_train.py > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc" > "$OUT/status.txt"; [ $rc -eq 0 ] || exit $rc
L=news_recommendation_project_v2_amd/libnewsrec_hip.so
timeout -k 10 400 python -u tools/gemm_ab.py --libs new=$L rb2=tools/gemm_lab/libnewsrec_rb2.so base=tools/gemm_lab/libnewsrec_base.so --rounds 5 \
  --shapes final,latent > "$OUT/gemm_ab.jsonl" 2> "$OUT/gemm_ab.err"
echo "gemm_ab rc=$?" >> "$OUT/status.txt"
