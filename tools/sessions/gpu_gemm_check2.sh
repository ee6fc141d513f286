# GEMM change check + A/B (current tree vs previous commit vs round-1 base) + stamps.
# Usage: bash tools/sessions/gpu_gemm_check2.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/gemm}
L=tools/gemm_lab
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_encoder.py tests/test_train.py > "$OUT/pytest_gemm.log" 2>&1 && \
timeout -k 10 600 python -u tools/gemm_ab.py --libs new=news_recommendation_project_v2_amd/libnewsrec_hip.so \
  cur=$L/libnewsrec_cur.so prev=$L/libnewsrec_prev.so > "$OUT/gemm_ab.jsonl" 2> "$OUT/gemm_ab.err" && \
timeout -k 10 300 python tools/gemm_lab/stamps.py > "$OUT/stamps.jsonl" 2> "$OUT/stamps.err"
