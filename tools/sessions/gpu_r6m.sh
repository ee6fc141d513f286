# round 6: do 128x256 half units on all 256 CUs beat 256x256 tiles on 132?
set -o pipefail
O=gpurun_out/r6m; mkdir -p $O
timeout -k 10 300 python -u tools/halves_probe.py --reps 50 --rounds 5 > $O/halves_probe.jsonl 2> $O/halves_probe.err
