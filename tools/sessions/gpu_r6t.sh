# round 6: latent step timeline after the dE-free token-LN grads
set -o pipefail
O=gpurun_out/r6t; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/tl_latent -o tl --output-format csv -- \
  python tools/train_bench.py --pooler latent --dtype bf16 --steps 12 > $O/tl_latent.json 2> $O/tl_latent.err || exit $?
f=$(find $O/tl_latent -name "*kernel_trace.csv" | head -1)
python tools/step_timeline.py $f > $O/latent_step_timeline.txt
