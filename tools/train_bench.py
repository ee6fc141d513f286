#!/usr/bin/env python3
"""Config-5 training-step throughput (BASELINE configs[4]: train_v3.py forward +
backward on 1x MI355X, bf16 MFMA backward).

Synthetic MIND-shaped batch: B training rows (one history group + one
positive + one negative each), history lengths ~ clip(geometric(1/33), 1, 600),
ids uniform over the news of the batch's impressions, token states N(0, 1)
last rows (only the last valid token reaches the token model).  Times
FinalAttentionTrainStep.step / LatentAttentionTrainStep.step (forward, backward, clip, AdamW) with HIP events
and prints one JSON line: rows/s, ms/step, MFMA TFLOP/s of the GEMMs.
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from news_recommendation_project_v2_amd import weights as W  # noqa: E402
from news_recommendation_project_v2_amd.modeling_utils import FinalAttention, get_token_attn_model  # noqa: E402
from news_recommendation_project_v2_amd.train_step import FinalAttentionTrainStep, TrainBatch  # noqa: E402


def make_batch(B: int, seed: int, dev):
    rng = np.random.default_rng(seed)
    h = np.clip(rng.geometric(1 / 33.0, B), 1, 600)
    ids = rng.integers(0, 40_000, int(h.sum()) + 2 * B)
    uniq, rev = np.unique(ids, return_inverse=True)
    Hs = int(h.sum())
    off = np.concatenate([[0], np.cumsum(h)]).astype(np.int64)
    tok = torch.randn((len(uniq), 1024), generator=torch.Generator().manual_seed(seed)).half()
    return TrainBatch(tok.to(dev), torch.as_tensor(rev[:Hs].astype(np.int32)).to(dev), torch.as_tensor(off).to(dev),
                      torch.as_tensor(rev[Hs:Hs + B].astype(np.int32)).to(dev),
                      torch.as_tensor(rev[Hs + B:].astype(np.int32)).to(dev)), Hs, len(uniq)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--dtype", choices=["bf16", "fp32"], default="bf16")
    ap.add_argument("--pooler", choices=["final", "latent"], default="final")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    dt = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    tm = get_token_attn_model()
    tm.load_state_dict(W.token_attn_state_dict(1234))
    if args.pooler == "latent":
        from news_recommendation_project_v2_amd.latent_attention import LatentAttentionModel
        from news_recommendation_project_v2_amd.train_step import LatentAttentionTrainStep
        lm = LatentAttentionModel()
        lm.load_state_dict(W.latent_attention_state_dict(1234))
        eng = LatentAttentionTrainStep(tm, lm.to(dev), dtype=dt, device=dev)
    else:
        fa = FinalAttention(1024, 4096)
        fa.load_state_dict(W.final_attention_state_dict(1234))
        eng = FinalAttentionTrainStep(tm, fa.to(dev), dtype=dt, device=dev)
    batch, Hs, U = make_batch(args.batch, 1234, dev)
    for _ in range(args.warmup):
        eng.step(batch)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    losses = [eng.step(batch) for _ in range(args.steps)]
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / args.steps
    fl = eng.flops_per_step(Hs)
    print(json.dumps({"metric": "config-5 training rows/s (fwd+bwd+clip+AdamW)", "dtype": args.dtype,
                      "batch_rows": args.batch, "history_slots": Hs, "unique_news": U, "ms_per_step": round(ms, 3),
                      "rows_per_s": round(args.batch / ms * 1e3, 1), "slots_per_s": round(Hs / ms * 1e3, 1),
                      "gemm_tflops": round(fl / ms / 1e9, 1),
                      "model_tflops_equiv": (round(eng.model_flops_per_step(Hs) / ms / 1e9, 1)
                                             if hasattr(eng, "model_flops_per_step") else None),
                      "loss_first": float(losses[0]),
                      "loss_last": float(losses[-1])}), flush=True)


if __name__ == "__main__":
    main()
