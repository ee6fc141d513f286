# round 6: pool_score PMC traffic passes (FETCH_SIZE / WRITE_SIZE / L2 hit-miss, one
# counter group per run) for the bench's roofline.traffic
set -uo pipefail
OUT=gpurun_out/r6j; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for cfg in "latent bf16" "final bf16"; do
  set -- $cfg
  for ctr in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
    tag=$(echo "$1_$2_$ctr" | tr ' ' '_')
    timeout -s KILL 90 rocprofv3 --pmc $ctr --kernel-include-regex pool_score -d "$OUT/pmc_$tag" -o pmc --output-format csv -- \
      python tools/profile_pool_score.py --pooler $1 --dtype $2 --reps 3 > "$OUT/pmc_$tag.log" 2>&1 || exit 2
  done
done
echo ok
