#!/usr/bin/env python3
"""A/B (tool only): bf16 latent transform, unfused (LN kernels + plain GEMMs)
vs LN-folded (nr_latent_transform_lnfold), interleaved in one process at
M = 72023; run under rocprofv3 --kernel-trace for per-kernel times."""
import json
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
from news_recommendation_project_v2_amd import ops  # noqa: E402
from news_recommendation_project_v2_amd import weights as W  # noqa: E402
from news_recommendation_project_v2_amd.latent_attention import LatentAttentionModel  # noqa: E402

dev = torch.device("cuda:0")
m = LatentAttentionModel()
m.load_state_dict(W.latent_attention_state_dict(1234))
m = m.to(dev).eval()
g = torch.Generator(device=dev).manual_seed(1234)
e = torch.randn((72023, 1024), generator=g, device=dev).to(torch.bfloat16)
wf = m.hip_weights(torch.bfloat16)
wu = {k: v for k, v in wf.items() if not k.endswith("_ln") and k not in ("ucq", "ucf")}
out = torch.empty_like(e)
res = {"fold": [], "unfused": []}
for _ in range(8):
    for tag, w in (("unfused", wu), ("fold", wf)):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ops.latent_transform(e, w, out=out)
        e0.record()
        for _ in range(5):
            ops.latent_transform(e, w, out=out)
        e1.record()
        torch.cuda.synchronize()
        res[tag].append(e0.elapsed_time(e1) / 5)
print(json.dumps({k: sorted(v) for k, v in res.items()}))
