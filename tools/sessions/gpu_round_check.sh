# Round check on the GPU box: gpu tests, smoke, bench, encoder bench, rocprof trace of the bench.
# Usage: bash tools/sessions/gpu_round_check.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/round}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build(); g.smoke()" > "$OUT/smoke.log" 2>&1 && \
timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" && \
timeout -k 10 300 python tools/encoder_bench.py > "$OUT/encoder_bench.log" 2>&1 && \
bash tools/prof_trace.sh "$OUT/prof"
