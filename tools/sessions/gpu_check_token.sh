set -o pipefail
mkdir -p gpurun_out/r1s2b
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/r1s2b/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python scripts/save_emb.py --synthetic --layers 2 --vocab 1000 --num-impressions 3000 --save-dir /tmp/emb > gpurun_out/r1s2b/save_emb.log 2>&1 && \
timeout -k 10 300 python scripts/save_emb.py --synthetic --layers 24 --vocab 250002 --dtype bf16 --num-impressions 20000 --splits MINDsmall_dev --save-dir /tmp/emb24 > gpurun_out/r1s2b/save_emb24.log 2>&1
