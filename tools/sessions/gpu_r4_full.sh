#!/bin/bash
# Round-4 full-tree check: smoke(), the whole -m gpu suite, the default bench line,
# the rocprof kernel-trace + PMC passes (tools/profile_round3.sh), and the
# M = 1.03 M, K = 4096 GEMM A/B against hipBLASLt.
set -o pipefail
OUT=gpurun_out/${1:-r4full}
mkdir -p "$OUT"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit 1
echo "smoke ok" > "$OUT/status.txt"
timeout -k 10 1000 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests \
  > "$OUT/pytest_gpu.log" 2>&1 || exit 2
echo "pytest ok" >> "$OUT/status.txt"
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 3
echo "bench ok" >> "$OUT/status.txt"
timeout -k 10 300 python -u tools/gemm_ab.py --m 1030000 --libs new=news_recommendation_project_v2_amd/libnewsrec_hip.so \
  --rounds 3 --reps 5 --shapes final.l3,latent.ff2 > "$OUT/gemm_ab_m1030000.jsonl" 2> "$OUT/gemm_ab_m1030000.err" || exit 4
echo "gemm_ab ok" >> "$OUT/status.txt"
timeout -k 10 300 python -u tools/gemm_ab.py --libs new=news_recommendation_project_v2_amd/libnewsrec_hip.so \
  --rounds 5 --shapes final,latent > "$OUT/gemm_ab.jsonl" 2> "$OUT/gemm_ab.err" || exit 5
echo "gemm_ab72k ok" >> "$OUT/status.txt"
bash tools/profile_round3.sh "$OUT/prof" > "$OUT/prof.log" 2>&1
echo "profile rc=$?" >> "$OUT/status.txt"
