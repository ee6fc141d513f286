#!/bin/bash
# Round-4: the N > 1 bench path on the one-GPU box (2 gloo ranks sharing the GPU:
# spawn, partition, sharded transform, host-staged all-gather, per-rank parity).
set -o pipefail
OUT=gpurun_out/${1:-r4dist}
mkdir -p "$OUT"
timeout -k 10 600 python -u bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 > "$OUT/bench_gloo2.json" 2> "$OUT/bench_gloo2.err"
echo "gloo2 rc=$?" > "$OUT/status.txt"
