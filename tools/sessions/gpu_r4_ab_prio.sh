#!/bin/bash
# Interleaved A/B of the latent step's side-stream priorities (NR_LT_PRIO: 0 default,
# 1 the fold-backward stream at the highest priority, 2 that plus the W1-grad stream at
# the lowest) on one box: train_bench.py latent bf16, 3 rounds x 3 settings.
# (The switch existed only for that run: no effect, not adopted.)
set -o pipefail
OUT=gpurun_out/${1:-r4ab}
mkdir -p "$OUT"
python - <<'PY' > "$OUT/prio_range.txt"
import ctypes
h = ctypes.CDLL("libamdhip64.so")
lo, hi = ctypes.c_int(), ctypes.c_int()
print("hipDeviceGetStreamPriorityRange", h.hipDeviceGetStreamPriorityRange(ctypes.byref(lo), ctypes.byref(hi)), lo.value, hi.value)
PY
for round in 1 2 3; do
  for v in 0 1 2; do
    NR_LT_PRIO=$v timeout -k 10 120 python -u tools/train_bench.py --pooler latent --dtype bf16 --steps 30 \
      > "$OUT/p${v}_r${round}.json" 2> "$OUT/p${v}_r${round}.err" || exit $?
    echo "p$v r$round $(cat $OUT/p${v}_r${round}.json)"
  done
done
