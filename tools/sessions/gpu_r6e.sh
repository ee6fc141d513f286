# round 6: the fold's small GEMMs alone (gemm64 vs the 256-tile grouped kernel)
set -o pipefail
O=gpurun_out/r6e; mkdir -p $O
timeout -k 10 300 python -u tools/gemm64_probe.py > $O/gemm64_probe.jsonl 2> $O/gemm64_probe.err || exit $?
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gemm_tn.py -k grouped64 > $O/pytest.log 2>&1
