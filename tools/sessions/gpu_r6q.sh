# round 6: persistent GEMM with the next tile's step-1 A1 DMA ahead of the epilogue and the
# first step's waits counted past the epilogue's stores (NR_GEMM_EARLY_A1): A/B + bitwise
# agreement on the transform shapes and the training M, then the whole GPU suite on that build
set -o pipefail
O=gpurun_out/r6q; mkdir -p $O
P=news_recommendation_project_v2_amd
L=tools/gemm_lab
timeout -k 10 600 python -u tools/gemm_ab.py --rounds 5 --libs new=$P/libnewsrec_hip.so ea1=$L/libnewsrec_ea1.so \
  > $O/gemm_ab.jsonl 2> $O/gemm_ab.err || exit $?
timeout -k 10 300 python -u tools/gemm_ab.py --m 8320 --rounds 5 --libs new=$P/libnewsrec_hip.so ea1=$L/libnewsrec_ea1.so \
  > $O/gemm_ab_8320.jsonl 2> $O/gemm_ab_8320.err || exit $?
cp $L/libnewsrec_ea1.so $P/libnewsrec_hip.so &&
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/ > $O/pytest_gpu_ea1.log 2>&1
