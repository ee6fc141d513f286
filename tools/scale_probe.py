#!/usr/bin/env python3
"""Probe (tool only): (1) per-news transform time vs shard rows (the per-rank
shard of an N-GPU strong-scaling run: 72023 / N rows), per GEMM kernel from
HIP events around each stage; (2) pool_score with the history and candidate
tables distinct (the bench: 2 x 147 MB > 256 MiB Infinity Cache) vs one shared
table, to price Infinity-Cache capacity.

    python tools/scale_probe.py > gpurun_out/probe/scale_probe.jsonl
"""
import json
import sys
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))

from news_recommendation_project_v2_amd import ops, synthetic  # noqa: E402
from news_recommendation_project_v2_amd import weights as W  # noqa: E402
from news_recommendation_project_v2_amd.engine import PoolScoreEngine  # noqa: E402
from news_recommendation_project_v2_amd.latent_attention import LatentAttentionModel  # noqa: E402


def ev_time(fn, reps=10):
    for _ in range(2):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    dev = torch.device("cuda:0")
    m = LatentAttentionModel()
    m.load_state_dict(W.latent_attention_state_dict(1234))
    m = m.to(dev).eval()
    n_news = 72023
    g = torch.Generator(device=dev).manual_seed(1234)
    table = torch.randn((n_news, 1024), generator=g, device=dev).to(torch.bfloat16)
    w = m.hip_weights(torch.bfloat16)
    for world in (1, 2, 4, 8):
        rows = (n_news + world - 1) // world
        src = table[:rows].contiguous()
        out = torch.empty_like(src)
        ws = torch.empty(64 << 20, dtype=torch.uint8, device=dev)
        need = None
        from news_recommendation_project_v2_amd import _lib
        need = _lib.load().nr_latent_workspace_bytes(_lib.NR_BF16, rows)
        ws = torch.empty(need, dtype=torch.uint8, device=dev)
        ms = ev_time(lambda: ops.latent_transform(src, w, out=out, workspace=ws))
        flop = rows * 2.0 * (1024 * 512 + 512 * 1024 + 1024 * 8192 + 4096 * 1024)
        print(json.dumps({"probe": "transform", "world": world, "rows": rows, "ms": round(ms, 4),
                          "tflops": round(flop / ms / 1e9, 1)}), flush=True)

    imps = synthetic.mind_impressions(n_news, 376471, seed=1234)
    eng = PoolScoreEngine(m, dtype=torch.bfloat16, device=dev).load_news(table.float())
    eng.load_impressions(imps.hist_idx, imps.hist_len, imps.cand_idx, imps.cand_len)
    eng.hist_table = eng.transform()
    eng.inv_norms()
    scores = torch.empty(imps.n_cand, dtype=torch.float32, device=dev)
    byt = imps.n_cand * (2048 + 12) + imps.n_hist * (2048 + 4) + imps.n_imp * 16
    ht = eng.hist_table
    for tag, h, c in [("distinct", ht, eng.cand_table), ("shared_cand", eng.cand_table, eng.cand_table),
                      ("shared_hist", ht, ht)]:
        inv = ops.row_inv_norm(c, 1e-8)
        f = lambda: ops.pool_score("latent", h, c, inv, eng.hist_idx, eng.hist_off, eng.cand_idx, eng.cand_off,
                                   imps.n_cand, scores=scores)
        ms = ev_time(f, 5)
        print(json.dumps({"probe": "pool_score", "tables": tag, "ms": round(ms, 4),
                          "GBs": round(byt / ms / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
