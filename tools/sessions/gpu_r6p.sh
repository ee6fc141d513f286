# round 6: FinalAttention step timeline on the final tree (K = 1024 GEMMs unsplit)
set -o pipefail
O=gpurun_out/r6p; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/tl_final -o tl --output-format csv -- \
  python tools/train_bench.py --pooler final --dtype bf16 --steps 12 > $O/tl_final.json 2> $O/tl_final.err || exit $?
f=$(find $O/tl_final -name "*kernel_trace.csv" | head -1)
python tools/step_timeline.py $f > $O/final_step_timeline.txt
