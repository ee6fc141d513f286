set -o pipefail
OUT=gpurun_out/s6b; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_encoder.py > $OUT/pytest_encoder.log 2>&1 && \
timeout -k 10 240 python -u tools/attn_ab.py --lab prev=tools/attnlab_tmp/lib_head.so early_w4=tools/attnlab_tmp/lib_enc_early_w4.so > $OUT/attn_ab.jsonl 2> $OUT/attn_ab.err && \
timeout -k 10 200 python -u tools/encoder_bench.py --n-news 16384 --dtype bf16 > $OUT/encoder_bench_len20.json 2> $OUT/encoder_bench_len20.err && \
timeout -k 10 200 python -u tools/encoder_bench.py --n-news 16384 --mean-len 66 --dtype bf16 > $OUT/encoder_bench_len66.json 2> $OUT/encoder_bench_len66.err
