#!/bin/bash
# Round-3 session 4: whole -m gpu suite (split tail now off by default, cut-invariance test),
# hipBLASLt kernel names / durations on the 8 transform shapes under rocprofv3, the default bench.
set -o pipefail
OUT=gpurun_out/${1:-r3s4b}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu ${TESTS:-tests} \
  > "$OUT/pytest_gpu.log" 2>&1 && \
( cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/gemm_trace" -o gemm --output-format csv -- \
  python tools/gemm_ab.py --rounds 3 --libs new=news_recommendation_project_v2_amd/libnewsrec_hip.so ${LABS:-} > "$OUT/gemm_ab.jsonl" 2> "$OUT/gemm_ab.err" ) && \
{ [ -z "${LABS:-}" ] || timeout -k 10 300 python -u tools/transform_ab.py --libs new=news_recommendation_project_v2_amd/libnewsrec_hip.so $LABS > "$OUT/transform_ab.jsonl" 2> "$OUT/transform_ab.err"; } && \
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
