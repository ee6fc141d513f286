#!/bin/bash
# Interleaved A/B/... of latent_train.hip variants on one box (source + library
# swapped together, since the loader checks the library's build hash against the
# sources): abtmp/latent_train.hip.V and abtmp/lib.V for each variant V, prepared
# in-tree first (build each variant, copy both files).  The tree is left on the
# first variant.  Usage: tools/ab_latent_variants.sh TAG [ROUNDS]
set -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT
P=news_recommendation_project_v2_amd
VARIANTS=$(ls abtmp | sed -n 's/^lib\.//p' | sort)
for i in $(seq 1 ${2:-3}); do
  for v in $VARIANTS; do
    cp abtmp/latent_train.hip.$v $P/csrc/latent_train.hip && cp abtmp/lib.$v $P/libnewsrec_hip.so || exit 9
    timeout -k 10 200 python -u tools/train_bench.py --pooler latent --dtype bf16 --steps 50 > $OUT/ab_${v}_$i.json 2> $OUT/ab_${v}_$i.err || exit $?
  done
done
first=$(echo $VARIANTS | cut -d' ' -f1)
cp abtmp/latent_train.hip.$first $P/csrc/latent_train.hip && cp abtmp/lib.$first $P/libnewsrec_hip.so
