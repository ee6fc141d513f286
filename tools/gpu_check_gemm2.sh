set -o pipefail
mkdir -p gpurun_out/gemm2
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -x -q > gpurun_out/gemm2/pytest_parity.log 2>&1 && \
NR_GEMM_MF16=1 timeout -k 10 600 python -m pytest tests/test_gpu_parity.py tests/test_train.py tests/test_encoder.py -m gpu -x -q -k "gemm or latent or train or encoder" > gpurun_out/gemm2/pytest_mf16.log 2>&1 && \
timeout -k 10 300 python tools/gemm_bench.py --dtypes bf16 > gpurun_out/gemm2/gemm_p32.log 2>&1 && \
NR_GEMM_MF16=1 timeout -k 10 300 python tools/gemm_bench.py --dtypes bf16 > gpurun_out/gemm2/gemm_p16.log 2>&1 && \
timeout -k 10 300 python tools/gemm_bench.py --dtypes bf16 > gpurun_out/gemm2/gemm_p32b.log 2>&1 && \
NR_GEMM_MF16=1 timeout -k 10 300 python tools/gemm_bench.py --dtypes bf16 > gpurun_out/gemm2/gemm_p16b.log 2>&1
