#!/bin/bash
# Round-3 s6: config-5 step wall time vs its summed kernel time (is the step launch-bound?):
# train_bench for both poolers, then a rocprofv3 kernel-trace of each (13 steps incl. warm-up).
set -o pipefail
OUT=gpurun_out/${1:-r3s6t}
mkdir -p "$OUT"
for P in final latent; do
  timeout -k 10 180 python -u tools/train_bench.py --pooler $P --steps 50 > "$OUT/train_$P.json" 2> "$OUT/train_$P.err" || exit 1
  ( cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
    timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/trace_$P" -o t --output-format csv -- \
    python tools/train_bench.py --pooler $P > "$OUT/train_${P}_prof.json" 2> "$OUT/train_${P}_prof.err" ) || exit 1
done
