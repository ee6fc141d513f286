#!/usr/bin/env python3
"""A/B (tool only): the bf16 per-news transforms with the split-K tail on and
off (nr_set_split_tail), interleaved in one process, median of rounds.

    python tools/split_tail_ab.py [--m 72023 9003] [--rounds 8]
"""
import argparse
import json
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from news_recommendation_project_v2_amd import _lib  # noqa: E402
from news_recommendation_project_v2_amd import weights as W  # noqa: E402
from news_recommendation_project_v2_amd.engine import PoolScoreEngine  # noqa: E402
from news_recommendation_project_v2_amd.latent_attention import LatentAttentionModel  # noqa: E402
from news_recommendation_project_v2_amd.modeling_utils import FinalAttention  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", nargs="+", type=int, default=[72023, 9003])
    ap.add_argument("--rounds", type=int, default=8)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    lib = _lib.load()
    for pooler in ("latent", "final"):
        m = LatentAttentionModel() if pooler == "latent" else FinalAttention(1024, 4096)
        m.load_state_dict(W.latent_attention_state_dict(1234) if pooler == "latent"
                          else W.final_attention_state_dict(1234))
        m = m.to(dev).eval()
        for n in args.m:
            g = torch.Generator(device=dev).manual_seed(n)
            table = torch.randn((n, 1024), generator=g, device=dev)
            eng = PoolScoreEngine(m, dtype=torch.bfloat16, device=dev).load_news(table)
            t = {0: [], 1: []}
            for _ in range(args.rounds):
                for on in (1, 0):
                    lib.nr_set_split_tail(on)
                    eng.hist_table = eng.transform(out=eng.hist_table)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(5):
                        eng.hist_table = eng.transform(out=eng.hist_table)
                    e1.record()
                    torch.cuda.synchronize()
                    t[on].append(e0.elapsed_time(e1) / 5)
            lib.nr_set_split_tail(0)
            print(json.dumps({"pooler": pooler, "m": n, "split_ms": round(float(np.median(t[1])), 4),
                              "nosplit_ms": round(float(np.median(t[0])), 4)}), flush=True)


if __name__ == "__main__":
    main()
