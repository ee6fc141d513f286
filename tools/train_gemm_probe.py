#!/usr/bin/env python3
"""Per-GEMM timing of the config-5 FinalAttention step's shapes at small M
(the training step's ~8.3k history slots) against the eval transform's M, to
see where the training GEMMs lose rate: tile rounds, epilogue, dropout hash.

    python tools/train_gemm_probe.py [--reps 30] [--ms 8192 8310 16384 72023]

Each line: shape, M, epilogue, µs per call (HIP events over --reps calls on
the current stream), TF/s; torch.matmul (hipBLASLt, no epilogue) beside it.
"""
import argparse
import json
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))

from news_recommendation_project_v2_amd import ops  # noqa: E402


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--ms", type=int, nargs="+", default=[8192, 8310, 16384, 72023])
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    for (K, N) in ((1024, 4096), (4096, 1024), (4096, 4096)):
        w = torch.randn(N, K, device=dev, generator=g).to(torch.bfloat16) * 0.03
        b = torch.randn(N, device=dev, generator=g) * 0.1
        for M in args.ms:
            a = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
            out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            fl = 2.0 * M * N * K
            cases = {
                "none": lambda: ops.gemm(a, w, b, "none", out=out),
                "relu": lambda: ops.gemm(a, w, b, "relu", out=out),
                "relu_dropout": lambda: ops.gemm_relu_dropout(a, w, b, 1234, 0.1, out=out),
                "drelu": lambda: ops.gemm_drelu(a, w, out, 1.1, out=torch.empty_like(out)),
                "hipblaslt": lambda: torch.matmul(a, w.t(), out=out),
            }
            for name, fn in cases.items():
                us = timed(fn, args.reps)
                print(json.dumps({"K": K, "N": N, "M": M, "epi": name, "us": round(us, 2),
                                  "tflops": round(fl / us / 1e6, 1)}), flush=True)
            del a, out
        del w, b


if __name__ == "__main__":
    main()
