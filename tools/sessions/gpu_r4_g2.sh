#!/bin/bash
# Round-4 GEMM session 2: balanced fragment reads (8/4/8/4) -- GEMM parity tests,
# then the per-shape A/B against the previous build (tools/gemm_lab/libnewsrec_base.so).
set -o pipefail
OUT=gpurun_out/${1:-r4g2}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gemm_half_tail.py tests/test_gemm_chunked.py tests/test_lnfold.py \
  "tests/test_gpu_parity.py::test_gemm_bf16_256_epilogues" "tests/test_gpu_parity.py::test_gemm_persistent_bf16_multi_tile" "tests/test_gpu_parity.py::test_gemm_persistent_inplace_resadd_ragged" \
  > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc" > "$OUT/status.txt"; [ $rc -eq 0 ] || exit $rc
L=news_recommendation_project_v2_amd/libnewsrec_hip.so
timeout -k 10 400 python -u tools/gemm_ab.py --libs new=$L rb=tools/gemm_lab/libnewsrec_rb.so base=tools/gemm_lab/libnewsrec_base.so --rounds 5 \
  --shapes final,latent > "$OUT/gemm_ab.jsonl" 2> "$OUT/gemm_ab.err"
echo "gemm_ab rc=$?" >> "$OUT/status.txt"
