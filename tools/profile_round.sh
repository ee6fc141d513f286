#!/bin/bash
# Round profile: kernel-trace stats of the headline bench + separate PMC passes
# (FETCH_SIZE, WRITE_SIZE, L2 hit/miss) on the pool+score kernel.
# Usage (on the GPU box): bash tools/profile_round.sh gpurun_out/prof_rNN
set -euo pipefail
OUT=${1:-gpurun_out/prof}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o bench --output-format csv -- \
  python bench.py --steps 10 --warmup 3 --no-extra --cpu-seconds 0 > "$OUT/bench_under_rocprof.json" 2> "$OUT/bench_under_rocprof.err"
for cfg in "latent bf16" "final bf16" "latent fp32"; do
  set -- $cfg
  for ctr in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
    tag=$(echo "$1_$2_$ctr" | tr ' ' '_')
    timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-include-regex pool_score -d "$OUT/pmc_$tag" -o pmc --output-format csv -- \
      python tools/profile_pool_score.py --pooler $1 --dtype $2 --reps 3 > "$OUT/pmc_$tag.log" 2>&1
  done
done
echo done
