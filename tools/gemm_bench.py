#!/usr/bin/env python3
"""Time the pooler-transform GEMM shapes (M = MIND-large news count) on the
HIP kernels; torch.matmul (hipBLASLt) is timed beside them as a yardstick only.

    python tools/gemm_bench.py [--m 72023]
"""
import argparse
import json
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from news_recommendation_project_v2_amd import ops  # noqa: E402

SHAPES = [  # (name, N, K, epilogue)
    ("final.l1 1024->4096 relu", 4096, 1024, "relu"),
    ("final.l2 4096->4096 relu", 4096, 4096, "relu"),
    ("final.l3 4096->1024", 1024, 4096, "none"),
    ("final.l5 4096->1024 exp", 1024, 4096, "exp"),
    ("latent.S 1024->512", 512, 1024, "none"),
    ("latent.B 512->1024 resadd", 1024, 512, "resadd"),
    ("latent.ff1 1024->8192 geglu", 8192, 1024, "geglu"),
    ("latent.ff2 4096->1024 resadd", 1024, 4096, "resadd"),
]


def timeit(fn, reps=10):
    for _ in range(2):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=72023)
    ap.add_argument("--dtypes", default="bf16,fp32")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    res = []
    for dts in args.dtypes.split(","):
        dt = torch.bfloat16 if dts == "bf16" else torch.float32
        for name, n, k, epi in SHAPES:
            a = (torch.randn(args.m, k, device=dev) * 0.1).to(dt)
            w = (torch.randn(n, k, device=dev) * 0.05).to(dt)
            b = torch.randn(n, device=dev) * 0.01
            ncols = n // 2 if epi == "geglu" else n
            out = torch.empty(args.m, ncols, device=dev, dtype=dt)
            r = torch.randn(args.m, ncols, device=dev).to(dt) if epi == "resadd" else None
            ms = timeit(lambda: ops.gemm(a, w, b, epilogue=epi, residual=r, out=out))
            ms_t = timeit(lambda: torch.matmul(a, w.T))
            tf = 2.0 * args.m * n * k / (ms * 1e-3) / 1e12
            res.append({"dtype": dts, "shape": name, "M": args.m, "N": n, "K": k, "ms": round(ms, 4),
                        "tflops": round(tf, 1), "torch_matmul_ms": round(ms_t, 4),
                        "torch_tflops": round(2.0 * args.m * n * k / (ms_t * 1e-3) / 1e12, 1)})
            print(json.dumps(res[-1]), flush=True)
    print(json.dumps({"summary": res}))


if __name__ == "__main__":
    main()
