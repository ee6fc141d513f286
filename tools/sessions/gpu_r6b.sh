# round 6: xfer / comm / training-parity GPU tests, then the PCIe probe
set -o pipefail
mkdir -p gpurun_out/r6b
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 180 --timeout-method thread -m gpu tests/test_xfer.py \
  tests/test_comm.py tests/test_train.py tests/test_latent_attention_autograd.py tests/test_final_attention_autograd.py \
  > gpurun_out/r6b/pytest.log 2>&1 &&
timeout -k 10 200 python -u tools/pcie_probe.py > gpurun_out/r6b/pcie.jsonl 2> gpurun_out/r6b/pcie.err
