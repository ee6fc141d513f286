#!/bin/bash
# Interleaved A/B/... of variants of one csrc file on one box (source + library
# swapped together, since the loader checks the library's build hash against the
# sources), timed by tools/train_bench.py.  abtmp/src.V (the variant's copy of the
# file) and abtmp/lib.V for each variant V are prepared in-tree first (build each
# variant, copy both).  The tree is left on the first variant.
# Usage: tools/ab_variants.sh TAG POOLER FILE [ROUNDS]   (FILE under csrc/, e.g. final_train.hip)
set -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT
P=news_recommendation_project_v2_amd
VARIANTS=$(ls abtmp | sed -n 's/^lib\.//p' | sort)
for i in $(seq 1 ${4:-3}); do
  for v in $VARIANTS; do
    cp abtmp/src.$v $P/csrc/$3 && cp abtmp/lib.$v $P/libnewsrec_hip.so || exit 9
    timeout -k 10 200 python -u tools/train_bench.py --pooler $2 --dtype bf16 --steps 50 > $OUT/ab_${v}_$i.json 2> $OUT/ab_${v}_$i.err || exit $?
  done
done
first=$(echo $VARIANTS | cut -d' ' -f1)
cp abtmp/src.$first $P/csrc/$3 && cp abtmp/lib.$first $P/libnewsrec_hip.so
