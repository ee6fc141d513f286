# Training-kernel check: GPU train tests, then the config-5 step with/without the grid-fill GEMM heuristic.
set -o pipefail
OUT=${1:-gpurun_out/train_check}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_train.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_train.log" 2>&1 && \
timeout -k 10 120 python tools/train_bench.py > "$OUT/train_bf16.json" 2>&1 && \
NR_GEMM_NO_AUTO_SMALL=1 timeout -k 10 120 python tools/train_bench.py > "$OUT/train_bf16_noauto.json" 2>&1 && \
timeout -k 10 120 python tools/train_bench.py --dtype fp32 > "$OUT/train_fp32.json" 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o train --output-format csv -- \
  python tools/train_bench.py > "$OUT/train_traced.log" 2>&1
