set -o pipefail
mkdir -p gpurun_out/gelu
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gelu/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python tools/gemm_bench.py --dtypes bf16,fp32 > gpurun_out/gelu/gemm.log 2>&1 && \
timeout -k 10 300 python tools/encoder_bench.py > gpurun_out/gelu/encoder.log 2>&1 && \
timeout -k 10 600 python bench.py > gpurun_out/gelu/bench.json 2> gpurun_out/gelu/bench.err
