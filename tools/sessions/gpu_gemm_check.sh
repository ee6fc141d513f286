# GEMM change check: GEMM / transform / encoder / training GPU tests, then the A/B timing.
# Usage: bash tools/sessions/gpu_gemm_check.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/gemm}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_encoder.py tests/test_train.py > "$OUT/pytest_gemm.log" 2>&1 && \
timeout -k 10 600 python -u tools/gemm_ab.py > "$OUT/gemm_ab.jsonl" 2> "$OUT/gemm_ab.err"
