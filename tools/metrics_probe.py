#!/usr/bin/env python3
"""Probe (tool only): dense ranks + MIND metrics kernels over the MIND-large-dev
shape (376 k impressions), HIP-event times per kernel.

    python tools/metrics_probe.py
"""
import json
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from news_recommendation_project_v2_amd import ops, synthetic  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    imps = synthetic.mind_shaped("mind_large_dev", seed=1234)
    s = torch.rand(imps.n_cand, device=dev)
    off = torch.as_tensor(imps.cand_off()).to(dev)
    y = torch.as_tensor(imps.labels.astype(np.float32)).to(dev)
    for _ in range(2):
        r = ops.dense_rank(s, off)
        ops.impression_metrics(r, y, off)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    t = np.zeros(2)
    for _ in range(10):
        ev[0].record()
        r = ops.dense_rank(s, off, check=False)
        ev[1].record()
        ops.impression_metrics(r, y, off)
        ev[2].record()
        torch.cuda.synchronize()
        t += [ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2])]
    print(json.dumps({"dense_rank_ms": round(t[0] / 10, 4), "impression_metrics_ms": round(t[1] / 10, 4),
                      "impressions": imps.n_imp, "candidates": imps.n_cand}))


if __name__ == "__main__":
    main()
