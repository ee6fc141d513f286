#!/usr/bin/env python3
"""Run the headline workload's kernels a few times for rocprofv3 counter passes.

    rocprofv3 --pmc FETCH_SIZE --kernel-include-regex pool_score -d OUT -- \
        python tools/profile_pool_score.py --pooler latent --dtype bf16

One transform + inverse-norm pass, then --reps pool+score launches on the
MIND-large-dev-shaped synthetic workload of bench.py.
"""
import argparse
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
from news_recommendation_project_v2_amd import synthetic  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pooler", default="latent", choices=["latent", "final"])
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--shape", default="mind_large_dev")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    n_news, n_imp = synthetic.SHAPES[args.shape]
    imps = synthetic.mind_impressions(n_news, n_imp, seed=1234)
    table = bench.news_table(n_news, dev)
    run = bench.Run(args.pooler, args.dtype, imps, table, dev, 0, 1)
    run.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.reps):
        run.eng.pool_score(scores=run.scores)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / args.reps * 1e3
    es = 2 if args.dtype == "bf16" else 4
    print(f"pool_score {args.pooler}/{args.dtype}: {ms:.3f} ms/launch (wall), algorithmic bytes/launch "
          f"{bench.ps_bytes(imps, args.pooler, es)}", flush=True)


if __name__ == "__main__":
    main()
