# round 6: interleaved A/B of the latent step's fold variants (NR_LT_FOLD64 0..3)
set -o pipefail
bash tools/ab_variants.sh r6f/ab latent latent_train.hip 3 || exit $?
O=gpurun_out/r6f; P=news_recommendation_project_v2_amd
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in v2; do
  cp abtmp/src.$v $P/csrc/latent_train.hip && cp abtmp/lib.$v $P/libnewsrec_hip.so || exit 9
  timeout -k 10 200 rocprofv3 --kernel-trace -d $O/tl_$v -o tl --output-format csv -- \
    python tools/train_bench.py --pooler latent --dtype bf16 --steps 12 > $O/tl_$v.json 2> $O/tl_$v.err || exit $?
  f=$(find $O/tl_$v -name "*kernel_trace.csv" | head -1)
  python tools/step_timeline.py $f > $O/timeline_$v.txt || exit $?
done
