#!/usr/bin/env python3
"""The FinalAttention step's N = 1024, K = 4096 GEMMs (linear3, linear5, dX) at
M = 8,320 padded slots: 132 tiles of 256x256 on 256 CUs leave half the chip idle
for one long round.  Times, in a HIP graph, the persistent kernel as the step
runs it against K-split layouts that fill the chip: the 8,192 main rows as two
K halves (256 half-length tiles), the 128 tail rows as `t` K-slices in the same
grouped launch, then one split-K fixup per part (main, tail); hipBLASLt beside.

    python tools/nsplit_probe.py [--reps 50]
"""
import argparse
import json
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))

from news_recommendation_project_v2_amd import ops  # noqa: E402
from tail_probe import timed  # noqa: E402


def cuts(K, n):
    """n K-slices of multiples of 64 summing to K."""
    q = K // 64
    return [64 * (q // n + (1 if i < q % n else 0)) for i in range(n)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    M, MM, N, K = 8320, 8192, 1024, 4096
    a = torch.randn(M, K, device=dev, generator=g).bfloat16()
    w = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).bfloat16()
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    ref = out.clone()
    res = {"persistent": timed(lambda: ops.gemm(a, w, out=out), args.reps)}
    ref.copy_(out)
    res["hipblaslt"] = timed(lambda: torch.matmul(a, w.t()), args.reps)
    for ms, ts in ((2, 2), (2, 4), (2, 6), (4, 4)):
        pm = torch.empty(ms, MM, N, device=dev)
        pt = torch.empty(ts, M - MM, N, device=dev)
        probs, k0 = [], 0
        for i, kk in enumerate(cuts(K, ms)):
            probs.append((a[:MM, k0:k0 + kk], w[:, k0:k0 + kk], pm[i]))
            k0 += kk
        k0 = 0
        for i, kk in enumerate(cuts(K, ts)):
            probs.append((a[MM:, k0:k0 + kk], w[:, k0:k0 + kk], pt[i]))
            k0 += kk

        def split(probs=probs, pm=pm, pt=pt):
            ops.gemm_grouped(probs)
            ops.splitk_fixup(pm, out[:MM], "none")
            ops.splitk_fixup(pt, out[MM:], "none")

        def gemm_only(probs=probs):
            ops.gemm_grouped(probs)
        res[f"split{ms}_tail{ts}"] = timed(split, args.reps)
        res[f"split{ms}_tail{ts}_gemm_only"] = timed(gemm_only, args.reps)
        err = float((out.float() - ref.float()).abs().max())
        res[f"split{ms}_tail{ts}_maxdiff_vs_persistent"] = err
    print(json.dumps({"M": M, "N": N, "K": K, "us": {k: round(v, 3) for k, v in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
