#!/bin/bash
# Round-3 s4: the threads/streams reentrancy test + cut-invariance test, then gloo N=2 and N=4
# rehearsals of bench.py's multi-rank path on the one GPU (sharded table vs overlapped build).
set -o pipefail
OUT=gpurun_out/${1:-r3s4g}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_gpu_parity.py::test_threads_on_their_own_streams_bit_identical" \
  "tests/test_gpu_parity.py::test_transform_rows_independent_of_the_cut" \
  "tests/test_gpu_parity.py::test_sharded_table_overlapped_rccl_single_rank" > "$OUT/pytest.log" 2>&1 && \
timeout -k 10 600 python -u bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 --cpu-seconds 0 \
  > "$OUT/bench_gloo2.json" 2> "$OUT/bench_gloo2.err" && \
timeout -k 10 600 python -u bench.py --gpus 4 --backend gloo --steps 3 --warmup 1 --cpu-seconds 0 \
  > "$OUT/bench_gloo4.json" 2> "$OUT/bench_gloo4.err"
