# round 6: latent step with dW1's last 256 rows K-sliced (no TN straggler tiles) vs the current step; then the latent tests on that build
set -o pipefail
O=gpurun_out/r6x; mkdir -p $O
P=news_recommendation_project_v2_amd
bash tools/ab_variants.sh r6x latent latent_train.hip 4 &&
cp abtmp/src.b_w1t $P/csrc/latent_train.hip && cp abtmp/lib.b_w1t $P/libnewsrec_hip.so &&
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_train.py \
  tests/test_latent_attention_autograd.py tests/test_train_bf16_drift.py > $O/pytest_latent.log 2>&1
