# round 6: round-end sequence after the latent token-LN grad change: smoke(), the full GPU suite, the default bench
set -o pipefail
O=gpurun_out/r6u; mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/ > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err
