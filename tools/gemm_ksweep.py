#!/usr/bin/env python3
"""K sweep of the bf16 256x256 GEMM at the latent ff1 shape (M = 72,023,
N = 8192): time(K) = fixed + per-K, so the per-tile fixed cost (prologue
fill + epilogue + block turnover) is the intercept.  Run once per kernel
variant (env NR_GEMM_PERSIST=1 selects the persistent kernel).

    python tools/gemm_ksweep.py [--m 72023] [--n 8192]
"""
import argparse
import json
import os
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from news_recommendation_project_v2_amd import ops  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
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
    ap.add_argument("--n", type=int, default=8192)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    variant = ("persistent" if os.environ.get("NR_GEMM_PERSIST") else "default") + f"-gm{os.environ.get('NR_GEMM_GROUP_M', 'default')}"
    tiles = ((args.m + 255) // 256) * (args.n // 256)
    rows = []
    for epi in ("none", "geglu"):
        for k in (512, 1024, 2048, 4096):
            a = (torch.randn(args.m, k, device=dev) * 0.1).to(torch.bfloat16)
            w = (torch.randn(args.n, k, device=dev) * 0.05).to(torch.bfloat16)
            b = torch.randn(args.n, device=dev) * 0.01
            out = torch.empty(args.m, args.n // 2 if epi == "geglu" else args.n, device=dev, dtype=torch.bfloat16)
            ms = timeit(lambda: ops.gemm(a, w, b, epilogue=epi, out=out))
            rows.append({"variant": variant, "epi": epi, "M": args.m, "N": args.n, "K": k, "ms": round(ms, 4),
                         "tflops": round(2.0 * args.m * args.n * k / (ms * 1e-3) / 1e12, 1)})
            print(json.dumps(rows[-1]), flush=True)
            del a, w, out
    for epi in ("none", "geglu"):
        ks = np.array([r["K"] for r in rows if r["epi"] == epi], dtype=float)
        ts = np.array([r["ms"] for r in rows if r["epi"] == epi])
        slope, icpt = np.polyfit(ks, ts, 1)
        waves = tiles / 256.0
        print(json.dumps({"variant": variant, "epi": epi, "fit_fixed_ms": round(icpt, 4),
                          "fit_ms_per_k1024": round(slope * 1024, 4),
                          "fixed_us_per_tile_round": round(icpt * 1e3 / np.ceil(waves), 2),
                          "tile_rounds": float(np.ceil(waves))}), flush=True)


if __name__ == "__main__":
    main()
