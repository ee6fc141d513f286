# Encoder check: GPU encoder tests, passage/query throughput, kernel traces.
set -o pipefail
OUT=${1:-gpurun_out/enc_check}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_encoder.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_encoder.log" 2>&1 && \
timeout -k 10 120 python tools/encoder_bench.py > "$OUT/enc_passage.json" 2>&1 && \
timeout -k 10 120 python tools/encoder_bench.py --mean-len 46 > "$OUT/enc_query.json" 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_q" -o encq --output-format csv -- \
  python tools/encoder_bench.py --mean-len 46 --reps 1 > "$OUT/enc_q_traced.log" 2>&1
