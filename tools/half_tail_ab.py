#!/usr/bin/env python3
"""A/B of the persistent GEMM's half-tile tail (nr_set_gemm_half_tail) on the
whole per-news transform at M = 72,023, both poolers, interleaved in one
process (guide §5.4 rule 24); the tables must be bit-identical.

    python tools/half_tail_ab.py [--n 72023] [--rounds 7] [--reps 10]
"""
import argparse
import json
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=72023)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    from news_recommendation_project_v2_amd import ops
    from news_recommendation_project_v2_amd import weights as W
    from news_recommendation_project_v2_amd.engine import PoolScoreEngine
    from news_recommendation_project_v2_amd.latent_attention import LatentAttentionModel
    from news_recommendation_project_v2_amd.modeling_utils import FinalAttention
    dev = torch.device("cuda:0")
    table = W.news_table(1234, args.n, 1024, name="half_tail_ab")
    for pooler in ("latent", "final"):
        m = LatentAttentionModel() if pooler == "latent" else FinalAttention(1024, 4096)
        m.load_state_dict(W.latent_attention_state_dict(1234) if pooler == "latent"
                          else W.final_attention_state_dict(1234))
        eng = PoolScoreEngine(m.to(dev).eval(), dtype=torch.bfloat16, device=dev).load_news(table)
        outs, times = {}, {"on": [], "off": []}
        for rnd in range(args.rounds):
            for lab in ("on", "off"):
                ops.set_gemm_half_tail(lab == "on")
                eng.transform()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.reps):
                    t = eng.transform()
                e1.record()
                torch.cuda.synchronize()
                times[lab].append(e0.elapsed_time(e1) / args.reps)
                if rnd == 0:
                    outs[lab] = t.clone()
        ops.set_gemm_half_tail(True)
        print(json.dumps({"pooler": pooler, "n": args.n,
                          **{f"{k}_ms": round(float(np.median(v)), 4) for k, v in times.items()},
                          **{f"{k}_min_ms": round(float(np.min(v)), 4) for k, v in times.items()},
                          "on_over_off": round(float(np.median(times["on"]) / np.median(times["off"])), 4),
                          "identical": bool(torch.equal(outs["on"], outs["off"]))}), flush=True)
        del eng, m


if __name__ == "__main__":
    main()
