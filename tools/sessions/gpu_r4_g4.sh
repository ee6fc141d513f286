#!/bin/bash
# Round-4 GEMM session 4: hand-off barrier inside the MFMA cluster (kHandoff 12
# shipped; 16 = round-start placement, 14, 8) -- GEMM parity tests, then the A/B.
set -o pipefail
OUT=gpurun_out/${1:-r4g4}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gemm_half_tail.py tests/test_gemm_chunked.py tests/test_lnfold.py \
  "tests/test_gpu_parity.py::test_gemm_bf16_256_epilogues" "tests/test_gpu_parity.py::test_gemm_persistent_bf16_multi_tile" \
  "tests/test_gpu_parity.py::test_gemm_persistent_inplace_resadd_ragged" > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc" > "$OUT/status.txt"; [ $rc -eq 0 ] || exit $rc
L=news_recommendation_project_v2_amd/libnewsrec_hip.so
G=tools/gemm_lab
timeout -k 10 500 python -u tools/gemm_ab.py --libs ho12=$L ho16=$G/libnewsrec_ho16.so ho14=$G/libnewsrec_ho14.so \
  ho8=$G/libnewsrec_ho8.so --rounds 5 --shapes final,latent > "$OUT/gemm_ab.jsonl" 2> "$OUT/gemm_ab.err"
echo "gemm_ab rc=$?" >> "$OUT/status.txt"
