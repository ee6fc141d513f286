set -o pipefail
mkdir -p gpurun_out/gemm
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gemm/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python tools/gemm_bench.py --dtypes bf16,fp32 > gpurun_out/gemm/gemm_p.log 2>&1 && \
NR_GEMM_V1=1 timeout -k 10 300 python tools/gemm_bench.py --dtypes bf16,fp32 > gpurun_out/gemm/gemm_v1.log 2>&1 && \
timeout -k 10 300 python bench.py --no-extra --cpu-seconds 0 > gpurun_out/gemm/bench.json 2> gpurun_out/gemm/bench.err
