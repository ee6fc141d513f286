# Kernel-trace stats of the headline bench (usage: bash tools/prof_trace.sh OUTDIR [bench args])
set -euo pipefail
OUT=${1:-gpurun_out/trace}
shift || true
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o bench --output-format csv -- \
  python bench.py --steps 10 --warmup 3 --no-extra --cpu-seconds 0 "$@" > "$OUT/bench_under_rocprof.json" 2> "$OUT/bench_under_rocprof.err"
find "$OUT/trace" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
