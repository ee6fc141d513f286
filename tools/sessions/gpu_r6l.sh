# round 6: lab A/B of staggered tile boundaries in the persistent GEMM (NR_GEMM_STAGGER)
set -o pipefail
O=gpurun_out/r6l; mkdir -p $O
L=tools/gemm_lab
timeout -k 10 600 python -u tools/gemm_ab.py --rounds 5 --libs new=news_recommendation_project_v2_amd/libnewsrec_hip.so \
  stg10=$L/libnewsrec_stg10.so stg20=$L/libnewsrec_stg20.so stg30=$L/libnewsrec_stg30.so > $O/gemm_ab.jsonl 2> $O/gemm_ab.err
