#!/bin/bash
# Round-4 session 2: the native latent config-5 step (nr_latent_train_step) and the
# round's new tests first, then the whole -m gpu suite, smoke, train benches (+ a
# rocprof kernel trace of the latent step), the default bench and the 2-rank gloo bench.
# Continues past test FAILURES (rc 1) but stops at anything else (fault, abort, timeout).
set -o pipefail
OUT=gpurun_out/${1:-r4s2}
mkdir -p "$OUT"
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 900 python -u -m pytest -v --timeout 900 --timeout-method thread -m gpu -s \
  tests/test_latent_attention_autograd.py tests/test_train_bf16_drift.py tests/test_comm.py tests/test_residency.py \
  > "$OUT/pytest_new.log" 2>&1
rc=$?; echo "new rc=$rc" > "$OUT/status.txt"; ok $rc || exit $rc
timeout -k 10 300 python -u tools/train_bench.py --pooler latent --dtype bf16 --steps 20 > "$OUT/train_latent_bf16.json" 2> "$OUT/train_latent_bf16.err"
rc=$?; echo "train latent rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || exit $rc
( cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_latent" -o tr --output-format csv -- \
  python tools/train_bench.py --pooler latent --dtype bf16 --steps 10 > "$OUT/train_latent_prof.json" 2> "$OUT/train_latent_prof.err" )
rc=$?; echo "rocprof rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest -v --timeout 600 --timeout-method thread -m gpu -s \
  --deselect tests/test_latent_attention_autograd.py --deselect tests/test_train_bf16_drift.py \
  --deselect tests/test_comm.py --deselect tests/test_residency.py tests/ > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "suite rc=$rc" >> "$OUT/status.txt"; ok $rc || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 && \
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" && \
timeout -k 10 400 python -u bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 --cpu-seconds 0 \
  > "$OUT/bench_gloo2.json" 2> "$OUT/bench_gloo2.err"
echo "tail rc=$?" >> "$OUT/status.txt"
