set -o pipefail
L=tools/gemm_lab
OUT=${1:-gpurun_out/ab}
mkdir -p $OUT
timeout -k 10 600 python -u tools/gemm_ab.py --shapes "${2:-}" --libs new=news_recommendation_project_v2_amd/libnewsrec_hip.so \
  ${3:-} > $OUT/gemm_ab.jsonl 2> $OUT/gemm_ab.err
