# GPU check of the tests added this session, then the full gpu suite and the default bench.
# Usage: bash tools/sessions/gpu_tests_new.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/new}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -s \
  tests/test_encoder.py tests/test_gpu_parity.py::test_pool_score_matches_reference_golden \
  tests/test_gpu_parity.py::test_gpu_f32_and_bf16_vs_oracle_auc tests/test_config2.py > "$OUT/pytest_new.log" 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 && \
timeout -k 10 900 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
