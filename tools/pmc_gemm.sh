set -euo pipefail
OUT=${1:-gpurun_out/pmc_gemm}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for shape in "8192 1024 geglu" "4096 4096 relu" "4096 1024 relu"; do
  set -- $shape
  tag="n$1_k$2_$3"
  mkdir -p "$OUT/$tag"
  for ctr in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY" "SQ_ACTIVE_INST_ANY SQ_INSTS_VALU" "GRBM_GUI_ACTIVE SQ_INSTS_MFMA" "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"; do
    ctag=$(echo "$ctr" | tr ' ' '_')
    timeout -k 10 120 rocprofv3 --pmc $ctr --kernel-include-regex gemm256 -d "$OUT/$tag/$ctag" -o pmc --output-format csv -- \
      python tools/profile_gemm.py $1 $2 $3 > "$OUT/$tag/$ctag.log" 2>&1
  done
done
echo done
