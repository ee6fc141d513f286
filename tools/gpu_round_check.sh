set -o pipefail
mkdir -p gpurun_out/r1s2
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/r1s2/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build(); g.smoke()" > gpurun_out/r1s2/smoke.log 2>&1 && \
timeout -k 10 600 python bench.py > gpurun_out/r1s2/bench.json 2> gpurun_out/r1s2/bench.err && \
timeout -k 10 300 python tools/encoder_bench.py > gpurun_out/r1s2/encoder_bench.log 2>&1
