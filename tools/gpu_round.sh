#!/bin/bash
# Round-5 GPU session.  Usage: tools/gpu_round.sh TAG STEP...
# Steps (run in the order given, each under its own timeout, stop at the first
# failure other than a test failure): drift, newtests, suite, smoke, bench, gloo2,
# trainprof, trainbench.
set -o pipefail
TAG=${1:-r5}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
for step in "$@"; do
  case $step in
    drift)
      timeout -k 10 600 python -u tools/drift_probe.py --pooler both --lr 1e-6 1e-4 > "$OUT/drift.jsonl" 2> "$OUT/drift.err"
      rc=$?; echo "drift rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || exit $rc ;;
    newtests)
      timeout -k 10 900 python -u -m pytest -v --timeout 900 --timeout-method thread -m gpu -s \
        tests/test_gemm_tn.py tests/test_train.py tests/test_train_bf16_drift.py tests/test_latent_attention_autograd.py tests/test_comm.py tests/test_gpu_parity.py > "$OUT/pytest_new.log" 2>&1
      rc=$?; echo "newtests rc=$rc" >> "$OUT/status.txt"; ok $rc || exit $rc ;;
    suite)
      timeout -k 10 1000 python -u -m pytest -v --timeout 600 --timeout-method thread -m gpu tests/ \
        > "$OUT/pytest_gpu.log" 2>&1
      rc=$?; echo "suite rc=$rc" >> "$OUT/status.txt"; ok $rc || exit $rc ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
      rc=$?; echo "smoke rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || exit $rc ;;
    bench)
      timeout -k 10 700 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
      rc=$?; echo "bench rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || exit $rc ;;
    gloo2)
      timeout -k 10 500 python -u bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 --cpu-seconds 0 \
        > "$OUT/bench_gloo2.json" 2> "$OUT/bench_gloo2.err"
      rc=$?; echo "gloo2 rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || exit $rc ;;
    trainbench)
      for p in final latent; do
        timeout -k 10 300 python -u tools/train_bench.py --pooler $p --dtype bf16 --steps 30 \
          > "$OUT/train_${p}_bf16.json" 2> "$OUT/train_${p}_bf16.err"
        rc=$?; echo "trainbench $p rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || exit $rc
      done ;;
    trainprof)
      for p in final latent; do
        ( cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
          timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_train_$p" -o tr --output-format csv -- \
          python tools/train_bench.py --pooler $p --dtype bf16 --steps 10 > "$OUT/train_${p}_prof.json" 2> "$OUT/train_${p}_prof.err" )
        rc=$?; echo "trainprof $p rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || exit $rc
      done ;;
    drifttest)
      timeout -k 10 1500 python -u -m pytest -v --timeout 1400 --timeout-method thread -m gpu -s \
        tests/test_train_bf16_drift.py > "$OUT/pytest_drift.log" 2>&1
      rc=$?; echo "drifttest rc=$rc" >> "$OUT/status.txt"; ok $rc || exit $rc ;;
    traintests)
      timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
        tests/test_train.py tests/test_gemm_tn.py tests/test_latent_attention_autograd.py > "$OUT/pytest_train.log" 2>&1
      rc=$?; echo "traintests rc=$rc" >> "$OUT/status.txt"; ok $rc || exit $rc ;;
    trainpmc)
      ( cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
        timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE \
        --kernel-include-regex gemm256 -d "$OUT/pmc_train_final" -o pmc --output-format csv -- \
        python tools/train_bench.py --pooler final --dtype bf16 --steps 4 > "$OUT/pmc_train_final.log" 2>&1 )
      rc=$?; echo "trainpmc rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || exit $rc ;;
    *) echo "unknown step $step" >> "$OUT/status.txt"; exit 2 ;;
  esac
done
