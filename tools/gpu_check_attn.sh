# Attention A/B: encoder GPU tests, then query/passage encoder throughput and kernel traces for the
# new build and the base build (NR_HIP_LIB) on the same box.  Usage: bash tools/gpu_check_attn.sh OUTDIR
set -o pipefail
OUT=$1
mkdir -p "$OUT"
BASE=$PWD/news_recommendation_project_v2_amd/libnewsrec_hip_base.so
timeout -k 10 300 python -u -m pytest tests/test_encoder.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_encoder.log" 2>&1 || exit 1
timeout -k 10 120 python tools/encoder_bench.py --mean-len 46 > "$OUT/enc_query.json" 2>&1 || exit 1
NR_HIP_LIB=$BASE timeout -k 10 120 python tools/encoder_bench.py --mean-len 46 > "$OUT/enc_query_base.json" 2>&1 || exit 1
timeout -k 10 120 python tools/encoder_bench.py > "$OUT/enc_passage.json" 2>&1 || exit 1
NR_HIP_LIB=$BASE timeout -k 10 120 python tools/encoder_bench.py > "$OUT/enc_passage_base.json" 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_q" -o encq --output-format csv -- python tools/encoder_bench.py --mean-len 46 --reps 1 > "$OUT/enc_q_traced.log" 2>&1
