#!/bin/bash
# Kernel trace of the FinalAttention config-5 step (train_bench.py --pooler final).
set -o pipefail
OUT=gpurun_out/${1:-r4ftr}
mkdir -p "$OUT"
( cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_final" -o tr --output-format csv -- \
  python tools/train_bench.py --pooler final --dtype bf16 --steps 10 > "$OUT/train_final_prof.json" 2> "$OUT/train_final_prof.err" )
echo "rocprof rc=$?" > "$OUT/status.txt"
