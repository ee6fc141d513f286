# round 6: FinalAttention step with the K = 1024 GEMMs unsplit (half-tile tail) vs the split-K tails; then its tests
set -o pipefail
O=gpurun_out/r6n; mkdir -p $O
P=news_recommendation_project_v2_amd
bash tools/ab_variants.sh r6n final final_train.hip 4 &&
cp abtmp/src.b_new $P/csrc/final_train.hip && cp abtmp/lib.b_new $P/libnewsrec_hip.so &&
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_train.py \
  tests/test_final_attention_autograd.py tests/test_train_bf16_drift.py > $O/pytest_final.log 2>&1
