# Default bench (with the PCIe extras) + tile-group sweep (gm 2 / 16) of the pooler GEMM shapes.
set -o pipefail
OUT=${1:-gpurun_out/fin}
mkdir -p "$OUT"
timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" && \
for g in 2 4 16; do
  NR_GEMM_GROUP_M=$g timeout -k 10 200 python tools/gemm_bench.py --dtypes bf16 > "$OUT/gemm_bench_gm$g.log" 2>&1 || exit 1
done
