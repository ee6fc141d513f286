# PMC passes on one big bf16 GEMM (M=262144, K=1024): N=4096 none / gelu.
set -uo pipefail
OUT=${1:-gpurun_out/pmc_gemm2}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for shape in "4096 1024 none" "4096 1024 gelu"; do
  set -- $shape
  tag="n$1_k$2_$3"; mkdir -p "$OUT/$tag"
  i=0
  for ctr in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS" \
             "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT" \
             "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $ctr --kernel-include-regex gemm256 -d "$OUT/$tag/p$i" -o pmc --output-format csv -- \
      python tools/profile_gemm.py $1 $2 $3 262144 > "$OUT/$tag/p$i.log" 2>&1 || echo "pass $tag $i failed rc=$?"
  done
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o tr --output-format csv -- python tools/profile_gemm.py 4096 1024 gelu 262144 > "$OUT/trace.log" 2>&1
echo done
