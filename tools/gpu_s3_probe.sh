# Bench with the new extras + kernel-trace breakdowns of the encoder and the config-5 train step.
set -o pipefail
OUT=${1:-gpurun_out/probe}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/enc" -o enc --output-format csv -- \
  python tools/encoder_bench.py --n-news 20000 --reps 2 > "$OUT/enc.log" 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/enc_q" -o encq --output-format csv -- \
  python tools/encoder_bench.py --n-news 20000 --reps 2 --mean-len 46 > "$OUT/enc_q.log" 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/train" -o train --output-format csv -- \
  python tools/train_bench.py > "$OUT/train.log" 2>&1
