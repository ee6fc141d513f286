# Full GPU check after a kernel change: all gpu tests, GEMM shapes at the pooler M and an
# encoder-sized M (new build, and the base build for A/B on the same box when present),
# encoder passage/query throughput, config-5 step, headline bench.
# Usage: bash tools/gpu_check_all.sh OUTDIR
set -o pipefail
OUT=$1
mkdir -p "$OUT"
BASE=$PWD/news_recommendation_project_v2_amd/libnewsrec_hip_base.so
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || exit 1
timeout -k 10 300 python tools/gemm_bench.py --dtypes bf16 > "$OUT/gemm_m72023.log" 2>&1 || exit 1
timeout -k 10 300 python tools/gemm_bench.py --dtypes bf16 --m 262144 > "$OUT/gemm_m262144.log" 2>&1 || exit 1
if [ -f "$BASE" ]; then
  NR_HIP_LIB=$BASE timeout -k 10 300 python tools/gemm_bench.py --dtypes bf16 > "$OUT/gemm_m72023_base.log" 2>&1 || exit 1
  NR_HIP_LIB=$BASE timeout -k 10 300 python tools/gemm_bench.py --dtypes bf16 --m 262144 > "$OUT/gemm_m262144_base.log" 2>&1 || exit 1
  NR_HIP_LIB=$BASE timeout -k 10 120 python tools/encoder_bench.py --mean-len 46 > "$OUT/enc_query_base.json" 2>&1 || exit 1
fi
timeout -k 10 120 python tools/encoder_bench.py > "$OUT/enc_passage.json" 2>&1 || exit 1
timeout -k 10 120 python tools/encoder_bench.py --mean-len 46 > "$OUT/enc_query.json" 2>&1 || exit 1
timeout -k 10 120 python tools/train_bench.py > "$OUT/train_bf16.json" 2>&1 || exit 1
timeout -k 10 600 python bench.py --cpu-seconds 5 > "$OUT/bench.json" 2> "$OUT/bench.err"
