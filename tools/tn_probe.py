#!/usr/bin/env python3
"""The latent step's weight-grad TN launch (dW1 = dG^T Y: M = 8,192, N = 1,024,
K = 8,320 slots, 128 tiles; dW2 = dm^T zbar: 64 tiles of K = 256) timed alone in a
HIP graph, to compare with its duration inside the step (beside the dY GEMM and
the row kernels on the other CUs).

    python tools/tn_probe.py [--reps 20]
"""
import argparse
import json
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "tools"))

from news_recommendation_project_v2_amd import ops  # noqa: E402
from tail_probe import timed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    Hp, F2, D, F, Bp = 8320, 8192, 1024, 4096, 256
    dG = torch.randn(Hp, F2, device=dev, generator=g).bfloat16()
    Y = torch.randn(Hp, D, device=dev, generator=g).bfloat16()
    dm = torch.randn(Bp, D, device=dev, generator=g).bfloat16()
    zb = torch.randn(Bp, F, device=dev, generator=g).bfloat16()
    gW1 = torch.empty(F2, D, device=dev)
    gW2 = torch.empty(D, F, device=dev)
    res = {"dW1_dW2": timed(lambda: ops.gemm_grouped_tn([(dG, Y, gW1), (dm, zb, gW2)]), args.reps),
           "dW1": timed(lambda: ops.gemm_grouped_tn([(dG, Y, gW1)]), args.reps),
           "dW1_as_2_row_halves": timed(lambda: ops.gemm_grouped_tn([(dG[:, :4096], Y, gW1[:4096]),
                                                                     (dG[:, 4096:], Y, gW1[4096:])]), args.reps)}
    fl = 2 * Hp * F2 * D
    print(json.dumps({"us": {k: round(v, 1) for k, v in res.items()}, "dW1_tflops": round(fl / res["dW1"] / 1e6, 1)}),
          flush=True)


if __name__ == "__main__":
    main()
