# round 6: GPU tests for xfer / comm / training parity / the 64-tile fold GEMM,
# an interleaved A/B of the latent step (a = round-5 fold chain, b = gemm64 fold),
# then the PCIe probe
set -o pipefail
O=gpurun_out/r6c; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -v -s --timeout 180 --timeout-method thread -m gpu tests/test_xfer.py \
  tests/test_comm.py tests/test_gemm_tn.py tests/test_train.py tests/test_latent_attention_autograd.py \
  tests/test_final_attention_autograd.py > $O/pytest.log 2>&1 || exit $?
bash tools/ab_variants.sh r6c/ab latent latent_train.hip 3 || exit $?
cp abtmp/src.b news_recommendation_project_v2_amd/csrc/latent_train.hip && cp abtmp/lib.b news_recommendation_project_v2_amd/libnewsrec_hip.so
timeout -k 10 200 python -u tools/pcie_probe.py > $O/pcie.jsonl 2> $O/pcie.err
