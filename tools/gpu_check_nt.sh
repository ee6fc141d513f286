# A/B: non-temporal GEMM epilogue stores (csrc/build_nt/libnewsrec_hip_nt.so via NR_HIP_LIB) vs the
# shipped stores, both with the grouped tile order; K sweep, pooler shapes, headline bench.
set -o pipefail
OUT=${1:-gpurun_out/nt}
mkdir -p "$OUT"
NT=$PWD/news_recommendation_project_v2_amd/csrc/build_nt/libnewsrec_hip_nt.so
export NR_GEMM_GROUP_M=4
NR_HIP_LIB=$NT timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k gemm > "$OUT/pytest_nt.log" 2>&1 && \
timeout -k 10 200 python tools/gemm_ksweep.py > "$OUT/ksweep_base.log" 2>&1 && \
NR_HIP_LIB=$NT timeout -k 10 200 python tools/gemm_ksweep.py > "$OUT/ksweep_nt.log" 2>&1 && \
timeout -k 10 200 python tools/gemm_bench.py --dtypes bf16,fp32 > "$OUT/gemm_bench_base.log" 2>&1 && \
NR_HIP_LIB=$NT timeout -k 10 200 python tools/gemm_bench.py --dtypes bf16,fp32 > "$OUT/gemm_bench_nt.log" 2>&1 && \
timeout -k 10 300 python bench.py --no-extra --cpu-seconds 0 > "$OUT/bench_base.json" 2> "$OUT/bench_base.err" && \
NR_HIP_LIB=$NT timeout -k 10 300 python bench.py --no-extra --cpu-seconds 0 > "$OUT/bench_nt.json" 2> "$OUT/bench_nt.err" && \
NR_GEMM_GROUP_M=1 timeout -k 10 300 python bench.py --no-extra --cpu-seconds 0 > "$OUT/bench_gm1.json" 2> "$OUT/bench_gm1.err"
