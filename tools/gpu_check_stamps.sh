# GEMM phase stamps (diagnostic build via NR_HIP_LIB) on the latent ff1 / ff2 / final l2 shapes.
set -o pipefail
OUT=${1:-gpurun_out/stamps}
mkdir -p "$OUT"
export NR_HIP_LIB=$PWD/news_recommendation_project_v2_amd/csrc/build_ab/libnewsrec_hip_stamps.so
timeout -k 10 120 python tools/gemm_stamps.py --n 8192 --k 1024 --epi geglu > "$OUT/ff1.json" 2> "$OUT/ff1.err" && \
timeout -k 10 120 python tools/gemm_stamps.py --n 8192 --k 1024 --epi none > "$OUT/ff1_none.json" 2> "$OUT/ff1_none.err" && \
timeout -k 10 120 python tools/gemm_stamps.py --n 8192 --k 4096 --epi none > "$OUT/k4096_none.json" 2> "$OUT/k4096.err" && \
timeout -k 10 120 python tools/gemm_stamps.py --n 1024 --k 4096 --epi none > "$OUT/ff2_none.json" 2> "$OUT/ff2.err"
