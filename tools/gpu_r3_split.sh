#!/bin/bash
# Split-K tail: equivalence tests + same-process A/B of the transforms, then the round-3 profile.
# A test assertion (pytest rc 1) does not stop the A/B; a timeout, abort or fault does.
set -o pipefail
OUT=gpurun_out/${1:-r3s}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_lnfold.py \
  "tests/test_gpu_parity.py::test_full_size_transform_vs_oracle" > "$OUT/pytest_split.log" 2>&1
rc=$?
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/split_tail_ab.py > "$OUT/split_tail_ab.jsonl" 2> "$OUT/split_tail_ab.err" && \
bash tools/profile_round3.sh "$OUT/prof"
