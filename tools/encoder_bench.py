#!/usr/bin/env python3
"""Title-encoder throughput (XLM-R-large shape, 24 layers, vocab 250,002) on
synthetic token ids shaped like MIND titles: passage ~ 20 +- 6 tokens, query
(QUERY_INSTRUCTION + title) ~ 46 +- 6 tokens.  Random weights
(speed does not depend on their values).  Reports news/s and tokens/s and the
MFMA fraction of the layer GEMMs.

    python tools/encoder_bench.py --n-news 20000 --dtype bf16
"""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from news_recommendation_project_v2_amd.encoder import XLMREncoder  # noqa: E402


def random_state_dict(dev, layers=24, vocab=250002):
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    r = lambda *s, sc=0.02: torch.randn(*s, generator=g, device=dev) * sc
    sd = {"embeddings.word_embeddings.weight": r(vocab, 1024), "embeddings.position_embeddings.weight": r(514, 1024),
          "embeddings.token_type_embeddings.weight": r(1, 1024),
          "embeddings.LayerNorm.weight": torch.ones(1024, device=dev),
          "embeddings.LayerNorm.bias": torch.zeros(1024, device=dev)}
    for i in range(layers):
        p = f"encoder.layer.{i}."
        for n in ("query", "key", "value"):
            sd[p + f"attention.self.{n}.weight"] = r(1024, 1024)
            sd[p + f"attention.self.{n}.bias"] = r(1024)
        sd[p + "attention.output.dense.weight"], sd[p + "attention.output.dense.bias"] = r(1024, 1024), r(1024)
        sd[p + "attention.output.LayerNorm.weight"] = torch.ones(1024, device=dev)
        sd[p + "attention.output.LayerNorm.bias"] = torch.zeros(1024, device=dev)
        sd[p + "intermediate.dense.weight"], sd[p + "intermediate.dense.bias"] = r(4096, 1024), r(4096)
        sd[p + "output.dense.weight"], sd[p + "output.dense.bias"] = r(1024, 4096), r(1024)
        sd[p + "output.LayerNorm.weight"] = torch.ones(1024, device=dev)
        sd[p + "output.LayerNorm.bias"] = torch.zeros(1024, device=dev)
    return sd


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-news", type=int, default=20000)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--mean-len", type=float, default=20.0)
    ap.add_argument("--reps", type=int, default=2)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    dt = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    enc = XLMREncoder(random_state_dict(dev), dtype=dt, device=dev, max_tokens=1 << 20)
    rng = np.random.default_rng(0)
    lens = np.clip(np.round(rng.normal(args.mean_len, 6, args.n_news)), 4, 512).astype(np.int64)
    ids = rng.integers(5, 250000, int(lens.sum())).astype(np.int32)
    enc.encode_packed(ids[:int(lens[:64].sum())], lens[:64])  # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.reps):
        enc.encode_packed(ids, lens)
    torch.cuda.synchronize()
    dt_s = (time.perf_counter() - t0) / args.reps
    T = int(lens.sum())
    flops = T * 24 * 2 * (3 * 1024 * 1024 + 1024 * 1024 + 2 * 1024 * 4096) + \
        float(24 * 4 * 1024 * (lens.astype(np.float64) ** 2).sum())
    print(json.dumps({"dtype": args.dtype, "n_news": args.n_news, "tokens": T, "mean_len": float(lens.mean()),
                      "seconds": round(dt_s, 4), "news_per_s": round(args.n_news / dt_s, 1),
                      "tokens_per_s": round(T / dt_s, 1), "tflops": round(flops / dt_s / 1e12, 1)}))


if __name__ == "__main__":
    main()
