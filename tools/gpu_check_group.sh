# A/B of the GEMM tile order (NR_GEMM_GROUP_M): parity tests under the grouped order, K sweep and
# pooler-shape bench for group 1 / 4 / 8.  Usage: bash tools/gpu_check_group.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/grp}
mkdir -p "$OUT"
NR_GEMM_GROUP_M=8 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k gemm > "$OUT/pytest_gm8.log" 2>&1 && \
NR_GEMM_GROUP_M=5 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k gemm > "$OUT/pytest_gm5.log" 2>&1 && \
for g in 1 4 8; do
  NR_GEMM_GROUP_M=$g timeout -k 10 200 python tools/gemm_ksweep.py > "$OUT/ksweep_gm$g.log" 2>&1 || exit 1
  NR_GEMM_GROUP_M=$g timeout -k 10 200 python tools/gemm_bench.py --dtypes bf16 > "$OUT/gemm_bench_gm$g.log" 2>&1 || exit 1
done
