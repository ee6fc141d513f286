# round 6: full GPU suite, then the default bench line (driver command)
set -o pipefail
O=gpurun_out/r6g; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/ > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err
