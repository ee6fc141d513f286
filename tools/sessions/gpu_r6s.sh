# round 6: latent step with the token-LN grads straight from the slots (no [U][1024] dE
# scatter, no ln_param_grad pass) vs the current step; then the latent / training tests
set -o pipefail
O=gpurun_out/r6s; mkdir -p $O
P=news_recommendation_project_v2_amd
bash tools/ab_variants.sh r6s latent latent_train.hip 4 &&
cp abtmp/src.b_new $P/csrc/latent_train.hip && cp abtmp/lib.b_new $P/libnewsrec_hip.so &&
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_train.py \
  tests/test_latent_attention_autograd.py tests/test_train_bf16_drift.py > $O/pytest_latent.log 2>&1
