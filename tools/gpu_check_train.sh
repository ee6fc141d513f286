set -o pipefail
mkdir -p gpurun_out/r1s2c
timeout -k 10 600 python -m pytest tests/test_train.py tests/test_token_attn.py -m gpu -x -q > gpurun_out/r1s2c/pytest_train.log 2>&1 && \
timeout -k 10 300 python tools/train_bench.py --dtype bf16 > gpurun_out/r1s2c/train_bench_bf16.json 2> gpurun_out/r1s2c/train_bench.err && \
timeout -k 10 300 python tools/train_bench.py --dtype fp32 > gpurun_out/r1s2c/train_bench_fp32.json 2>> gpurun_out/r1s2c/train_bench.err && \
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/r1s2c/pytest_gpu_all.log 2>&1 && \
timeout -k 10 300 python scripts/save_emb.py --synthetic --layers 2 --vocab 1000 --num-impressions 3000 --save-dir /tmp/emb > gpurun_out/r1s2c/save_emb.log 2>&1 && \
timeout -k 10 300 python scripts/save_emb.py --synthetic --layers 24 --vocab 250002 --dtype bf16 --num-impressions 20000 --splits MINDsmall_dev --save-dir /tmp/emb24 > gpurun_out/r1s2c/save_emb24.log 2>&1
