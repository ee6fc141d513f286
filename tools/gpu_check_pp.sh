set -o pipefail
mkdir -p gpurun_out/pp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pp/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python tools/gemm_bench.py --dtypes bf16 > gpurun_out/pp/gemm_pp.log 2>&1 && \
NR_GEMM_NOPERSIST=1 timeout -k 10 300 python tools/gemm_bench.py --dtypes bf16 > gpurun_out/pp/gemm_p16.log 2>&1 && \
timeout -k 10 300 python tools/encoder_bench.py > gpurun_out/pp/encoder.log 2>&1 && \
timeout -k 10 600 python bench.py --cpu-seconds 0 > gpurun_out/pp/bench.json 2> gpurun_out/pp/bench.err
