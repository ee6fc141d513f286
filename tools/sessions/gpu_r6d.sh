# round 6: (1) one-step kernel timelines of the latent config-5 step, variant a
# (round-5 fold chain) and b (gemm64 fold), to see where b lost; (2) the transform
# GEMMs' clock: in-kernel s_memtime / s_memrealtime after 2 s of
# back-to-back launches (stamped diagnostic build), and GRBM_GUI_ACTIVE / 8 over the
# kernel-trace duration (one rocprofv3 pass per shape, 20 launches)
set -o pipefail
O=gpurun_out/r6d; mkdir -p $O
P=news_recommendation_project_v2_amd
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in a b; do
  cp abtmp/src.$v $P/csrc/latent_train.hip && cp abtmp/lib.$v $P/libnewsrec_hip.so || exit 9
  timeout -k 10 200 rocprofv3 --kernel-trace -d $O/tl_$v -o tl --output-format csv -- \
    python tools/train_bench.py --pooler latent --dtype bf16 --steps 12 > $O/tl_$v.json 2> $O/tl_$v.err || exit $?
  f=$(find $O/tl_$v -name "*kernel_trace.csv" | head -1)
  python tools/step_timeline.py $f > $O/timeline_$v.txt || exit $?
done
cp abtmp/src.b $P/csrc/latent_train.hip && cp abtmp/lib.b $P/libnewsrec_hip.so
timeout -k 10 300 python -u tools/gemm_lab/stamps.py > $O/stamps.jsonl 2> $O/stamps.err || exit $?
for shape in "8192 1024 geglu" "4096 4096 relu" "1024 4096 none" "512 1024 softmax64" "1024 512 resadd"; do
  set -- $shape
  tag="n$1_k$2_$3"
  timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --kernel-trace --stats --kernel-include-regex gemm256 \
    -d $O/clk_$tag -o clk --output-format csv -- python tools/profile_gemm.py $1 $2 $3 72023 20 > $O/clk_$tag.log 2>&1 || exit $?
done
echo ok
