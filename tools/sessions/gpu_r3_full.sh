#!/bin/bash
# Round-3 full check: the whole -m gpu suite, the default bench line, then the rocprof
# kernel-trace + PMC passes of tools/profile_round3.sh.  Usage: bash tools/sessions/gpu_r3_full.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-r3full}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
  > "$OUT/pytest_gpu.log" 2>&1 && \
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" && \
bash tools/profile_round3.sh "$OUT/prof"
