#!/bin/bash
# Round-3 s4: latent-attention training tests (module autograd, train step f32 / bf16, train_v3 --pooler latent)
# and the config-5 trainer tests, then the default bench (incl. the latent training leg).
set -o pipefail
OUT=gpurun_out/${1:-r3lat3}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_latent_attention_autograd.py \
  tests/test_final_attention_autograd.py > "$OUT/pytest.log" 2>&1 && \
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
