#!/bin/bash
# Interleaved A/B of the latent step's stream layouts (NR_LT_VARIANT 0 / 1 / 2) on one
# box: train_bench.py latent bf16, 3 rounds x 3 variants, one JSON line each.
# (The switch existed only for that run; layout 2 is the product now.)
set -o pipefail
OUT=gpurun_out/${1:-r4ab}
mkdir -p "$OUT"
for round in 1 2 3; do
  for v in 0 1 2; do
    NR_LT_VARIANT=$v timeout -k 10 120 python -u tools/train_bench.py --pooler latent --dtype bf16 --steps 30 \
      > "$OUT/v${v}_r${round}.json" 2> "$OUT/v${v}_r${round}.err" || exit $?
    echo "v$v r$round $(cat $OUT/v${v}_r${round}.json)"
  done
done
