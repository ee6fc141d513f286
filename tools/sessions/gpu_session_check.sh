# GPU check of the current tree: gpu tests, smoke, default bench, 2-rank (gloo) bench spawn.
# Usage: bash tools/sessions/gpu_session_check.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/check}
mkdir -p "$OUT"
python -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count(), 'omp', os.environ.get('OMP_NUM_THREADS'))" > "$OUT/host.txt"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 && \
timeout -k 10 900 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" && \
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --no-extra --steps 3 --warmup 1 > "$OUT/bench_gloo2.json" 2> "$OUT/bench_gloo2.err"
