#!/bin/bash
# Round-3 profile on the GPU box (same recipe as tools/profile_round2.sh):
#  1. rocprofv3 --kernel-trace --stats of the headline bench (no extras, no CPU leg, no AUC gate)
#  2. PMC passes on pool_score_kernel (FETCH_SIZE / WRITE_SIZE / L2 hit-miss), one counter group per run
#  3. MFMA-busy PMC passes on the persistent GEMM (latent ff1 GEGLU and final.l2 shapes, M = 72,023)
# Usage: bash tools/profile_round3.sh gpurun_out/prof_r3
set -uo pipefail
OUT=${1:-gpurun_out/prof_r3}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o bench --output-format csv -- \
  python bench.py --steps 10 --warmup 3 --no-extra --cpu-seconds 0 > "$OUT/bench_under_rocprof.json" 2> "$OUT/bench_under_rocprof.err" || exit 1
for cfg in "latent bf16" "final bf16"; do
  set -- $cfg
  for ctr in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
    tag=$(echo "$1_$2_$ctr" | tr ' ' '_')
    timeout -s KILL 90 rocprofv3 --pmc $ctr --kernel-include-regex pool_score -d "$OUT/pmc_$tag" -o pmc --output-format csv -- \
      python tools/profile_pool_score.py --pooler $1 --dtype $2 --reps 3 > "$OUT/pmc_$tag.log" 2>&1 || exit 2
  done
done
SQ1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS"
SQ2="SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT"
for shape in "8192 1024 geglu" "4096 4096 relu"; do
  set -- $shape
  tag="gemm_n$1_k$2_$3"; mkdir -p "$OUT/$tag"
  i=0
  for ctr in "$SQ1" "$SQ2" "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $ctr --kernel-include-regex gemm256t -d "$OUT/$tag/p$i" -o pmc --output-format csv -- \
      python tools/profile_gemm.py $1 $2 $3 72023 > "$OUT/$tag/p$i.log" 2>&1 || exit 3
  done
done
echo done
