# A/B: bf16 epilogue slab (shipped) vs f32 slab
# (csrc/build_ab/libnewsrec_hip_ab.so, -DNR_GEMM_SLAB16=0, via NR_HIP_LIB).
set -o pipefail
OUT=${1:-gpurun_out/slab16}
mkdir -p "$OUT"
AB=$PWD/news_recommendation_project_v2_amd/csrc/build_ab/libnewsrec_hip_ab.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_train.py tests/test_encoder.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 && \
timeout -k 10 200 python tools/gemm_ksweep.py > "$OUT/ksweep_new.log" 2>&1 && \
NR_HIP_LIB=$AB timeout -k 10 200 python tools/gemm_ksweep.py > "$OUT/ksweep_base.log" 2>&1 && \
timeout -k 10 200 python tools/gemm_bench.py --dtypes bf16 > "$OUT/gemm_bench_new.log" 2>&1 && \
NR_HIP_LIB=$AB timeout -k 10 200 python tools/gemm_bench.py --dtypes bf16 > "$OUT/gemm_bench_base.log" 2>&1 && \
timeout -k 10 300 python bench.py --no-extra --cpu-seconds 0 > "$OUT/bench_new.json" 2> "$OUT/bench_new.err" && \
NR_HIP_LIB=$AB timeout -k 10 300 python bench.py --no-extra --cpu-seconds 0 > "$OUT/bench_base.json" 2> "$OUT/bench_base.err" && \
timeout -k 10 300 python tools/encoder_bench.py > "$OUT/encoder_new.log" 2>&1 && \
NR_HIP_LIB=$AB timeout -k 10 300 python tools/encoder_bench.py > "$OUT/encoder_base.log" 2>&1
