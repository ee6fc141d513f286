# round 6: rehearsal of the N > 1 bench on the one-GPU box with the round-6 launcher
# (gloo: two ranks share the GPU; RCCL needs a GPU per rank): the self-spawning form
# (spawn_ranks, phase records) and the driver's torch.distributed.run form
set -o pipefail
O=gpurun_out/r6r; mkdir -p $O
timeout -k 10 600 python -u bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 --no-cpu-10k --cpu-seconds 0 \
  --no-auc-gate > $O/bench_gloo2_spawn.json 2> $O/bench_gloo2_spawn.err || exit $?
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 --no-cpu-10k --cpu-seconds 0 \
  --no-auc-gate > $O/bench_gloo2_torchrun.json 2> $O/bench_gloo2_torchrun.err
