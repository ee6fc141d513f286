#!/bin/bash
# Round-4 session g7: residual rows 0-1 issued in the last K step -- RESADD /
# SOFTMAX64_BWD parity tests and the A/B against the previous build.
set -o pipefail
OUT=gpurun_out/${1:-r4g7}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu \
  tests/test_gemm_half_tail.py tests/test_gemm_chunked.py "tests/test_gpu_parity.py::test_gemm_bf16_256_epilogues" \
  "tests/test_gpu_parity.py::test_gemm_persistent_bf16_multi_tile" "tests/test_gpu_parity.py::test_gemm_persistent_inplace_resadd_ragged" \
  tests/test_latent_attention_autograd.py tests/test_train.py > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc" > "$OUT/status.txt"; [ $rc -eq 0 ] || exit $rc
L=news_recommendation_project_v2_amd/libnewsrec_hip.so
timeout -k 10 300 python -u tools/gemm_ab.py --libs new=$L pre=tools/gemm_lab/libnewsrec_pre.so --rounds 7 \
  --shapes latent.B,latent.ff2,final.l3 > "$OUT/gemm_ab.jsonl" 2> "$OUT/gemm_ab.err"
echo "gemm_ab rc=$?" >> "$OUT/status.txt"
timeout -k 10 300 python -u tools/gemm_ab.py --m 1030000 --libs new=$L pre=tools/gemm_lab/libnewsrec_pre.so \
  --rounds 3 --reps 5 --shapes latent.ff2 > "$OUT/gemm_ab_m1030000.jsonl" 2> "$OUT/gemm_ab_m1030000.err"
echo "gemm_ab_1m rc=$?" >> "$OUT/status.txt"
