#!/bin/bash
# Round-4 session 3: native latent step v2 (parallel fold backward, contiguous atomics,
# side stream for the W1 weight grad) -- its tests, the bf16 drift test, the comm test,
# then the train bench and a rocprof kernel trace of the latent step.
set -o pipefail
OUT=gpurun_out/${1:-r4s3}
mkdir -p "$OUT"
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 900 python -u -m pytest -v --timeout 900 --timeout-method thread -m gpu -s \
  tests/test_latent_attention_autograd.py tests/test_train_bf16_drift.py tests/test_comm.py tests/test_train.py \
  > "$OUT/pytest_new.log" 2>&1
rc=$?; echo "new rc=$rc" > "$OUT/status.txt"; ok $rc || exit $rc
timeout -k 10 300 python -u tools/train_bench.py --pooler latent --dtype bf16 --steps 20 > "$OUT/train_latent_bf16.json" 2> "$OUT/train_latent_bf16.err"
rc=$?; echo "train latent rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/train_bench.py --pooler final --dtype bf16 --steps 20 > "$OUT/train_final_bf16.json" 2> "$OUT/train_final_bf16.err"
rc=$?; echo "train final rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || exit $rc
( cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_latent" -o tr --output-format csv -- \
  python tools/train_bench.py --pooler latent --dtype bf16 --steps 10 > "$OUT/train_latent_prof.json" 2> "$OUT/train_latent_prof.err" )
echo "rocprof rc=$?" >> "$OUT/status.txt"
