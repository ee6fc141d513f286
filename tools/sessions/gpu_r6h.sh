# round 6: the tightened parity tests with their printed ratios, the default bench line,
# and the rocprofv3 kernel-trace summary of the headline (profiles/round6/final)
set -o pipefail
O=gpurun_out/r6h; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_latent_attention_autograd.py tests/test_final_attention_autograd.py tests/test_train.py \
  tests/test_api_end_to_end.py tests/test_comm.py > $O/pytest.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
bash tools/prof_trace.sh $O/prof
