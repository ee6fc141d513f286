#!/usr/bin/env python3
"""VERDICT r5 #3's question for the FinalAttention step's N = 1024 GEMMs
(linear3, linear5, dX: K = 4096): would 128 x 256 output units that fill all
256 CUs beat 256 x 256 tiles that fill 132 of them?  The persistent kernel
already has such a unit -- the half tile of its last partial round (wave group
0 computes rows mb .. mb + 127 of a 256-wide column block with the full-tile K
chain) -- so the probe needs no new kernel: at M = 8,192 the 128 tiles are cut
into 256 halves (one round, every CU) when the half tail is on, and run as 128
full tiles when it is off.  M = 8,320 (the benchmark batch's padded slots) is
timed as the step runs it (132 full tiles) and as 256 halves over the first
8,192 rows plus the 128 tail rows as K-slices + fixup (the step's own tail form
for its N = 4096 GEMMs).  Also the K = 1024, N = 4096 shape (linear1 / linear4 /
dY / dZ2) for the same cut.  HIP-graph timing, interleaved rounds, medians.

    python tools/halves_probe.py [--reps 50] [--rounds 5]
"""
import argparse
import json
import statistics
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "tools"))

from news_recommendation_project_v2_amd import ops  # noqa: E402
from tail_probe import timed  # noqa: E402


def cuts(K, n):
    q = K // 64
    return [64 * (q // n + (1 if i < q % n else 0)) for i in range(n)]


def shape(N, K, reps, rounds, dev):
    g = torch.Generator(device=dev).manual_seed(0)
    M, MM = 8320, 8192
    a = torch.randn(M, K, device=dev, generator=g).bfloat16()
    w = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).bfloat16()
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    ref = torch.empty_like(out)
    ts = 4 if K <= 1024 else 8
    pt = torch.empty(ts, M - MM, N, device=dev)
    tail = []
    k0 = 0
    for i, kk in enumerate(cuts(K, ts)):
        tail.append((a[MM:, k0:k0 + kk], w[:, k0:k0 + kk], pt[i]))
        k0 += kk

    def full8320():
        ops.set_gemm_half_tail(True)  # 132 tiles on 256 CUs: no cut (264 halves > 256)
        ops.gemm(a, w, out=out)

    def halves8192():
        ops.set_gemm_half_tail(True)
        ops.gemm(a[:MM], w, out=out[:MM])

    def full8192():
        ops.set_gemm_half_tail(False)
        ops.gemm(a[:MM], w, out=out[:MM])

    def halves_plus_tail():
        ops.set_gemm_half_tail(True)
        ops.gemm(a[:MM], w, out=out[:MM])
        ops.gemm_grouped(tail)
        ops.splitk_fixup(pt, out[MM:], "none")

    variants = {"full_8320": full8320, "halves_8192": halves8192, "full_8192": full8192,
                "halves_8192_plus_tail_8320": halves_plus_tail}
    t = {k: [] for k in variants}
    for _ in range(rounds):
        for k, fn in variants.items():
            t[k].append(timed(fn, reps))
    ops.set_gemm_half_tail(True)
    full8320()
    torch.cuda.synchronize()
    ref.copy_(out)
    halves_plus_tail()
    torch.cuda.synchronize()
    diff = float((out.float() - ref.float()).abs().max())
    flop = 2.0 * N * K
    med = {k: statistics.median(v) for k, v in t.items()}
    rec = {"N": N, "K": K, "us": {k: round(v, 2) for k, v in med.items()},
           "us_all": {k: [round(x, 2) for x in v] for k, v in t.items()},
           "tflops": {k: round(flop * (M if k.endswith("8320") else MM) / (v * 1e-6) / 1e12, 1) for k, v in med.items()},
           "maxdiff_halves_plus_tail_vs_full": diff}
    print(json.dumps(rec), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=5)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    for N, K in ((1024, 4096), (4096, 1024)):
        shape(N, K, args.reps, args.rounds, dev)
    ops.set_gemm_half_tail(True)


if __name__ == "__main__":
    main()
