#!/bin/bash
# Round-3 final-tree check: smoke(), the whole -m gpu suite, the default bench line, and the
# rocprof kernel-trace + PMC passes (tools/profile_round3.sh).
set -o pipefail
OUT=gpurun_out/${1:-r3final}
mkdir -p "$OUT"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 && \
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
  > "$OUT/pytest_gpu.log" 2>&1 && \
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" && \
bash tools/profile_round3.sh "$OUT/prof"
