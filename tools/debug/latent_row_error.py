#!/usr/bin/env python3
"""Debug (tool only): stage-by-stage bf16 vs f32 error of the latent transform
chain for the worst row (tests/test_lnfold.py inputs)."""
import sys
from pathlib import Path
import torch
REPO = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(REPO))
from news_recommendation_project_v2_amd import ops  # noqa: E402
from news_recommendation_project_v2_amd import weights as W  # noqa: E402
from news_recommendation_project_v2_amd.latent_attention import LatentAttentionModel  # noqa: E402

dev = torch.device("cuda:0")
m = LatentAttentionModel(); m.load_state_dict(W.latent_attention_state_dict(1234, ln_random=True)); m = m.to(dev).eval()
n = 300
g = torch.Generator().manual_seed(n)
e = (torch.randn(n, 1024, generator=g) * 0.8 + torch.randn(n, 1, generator=g) * 0.5).to(torch.bfloat16).to(dev)
fw = {k: v.to(dev) for k, v in m.folded_weights().items()}
x = e.double()
def chain(x, P_round=None):
    y = torch.nn.functional.layer_norm(x, (1024,), fw["lnq_g"], fw["lnq_b"], 1e-5)
    s = y @ fw["A"].T
    p = torch.softmax(s.reshape(-1, 8, 64), -1).reshape(-1, 512)
    h1 = x + p @ fw["Bt"].T
    z = torch.nn.functional.layer_norm(h1, (1024,), fw["lnf_g"], fw["lnf_b"], 1e-5) @ fw["W1i"].T + fw["b1i"]
    z = z.reshape(-1, 128, 2, 32)
    f = (z[:, :, 0] * torch.nn.functional.gelu(z[:, :, 1])).reshape(-1, 4096)
    return dict(s=s, p=p, h1=h1, z=z, f=f, h=h1 + f @ fw["W2"].T + fw["b2"])
ref = chain(x)
out16 = ops.latent_transform(e, m.hip_weights(torch.bfloat16)).double()
out32 = ops.latent_transform(e.float(), m.hip_weights(torch.float32)).double()
e16 = (out16 - ref["h"]).abs().max(1).values; e32 = (out32 - ref["h"]).abs().max(1).values
r = int(e16.argmax())
print("worst row", r, "err16", e16[r].item(), "err32", e32[r].item(), "median err16", e16.median().item())
print("max |s| row", ref["s"][r].abs().max().item(), "max p", ref["p"][r].max().item())
print("max |z| row", ref["z"][r].abs().max().item(), "max |f|", ref["f"][r].abs().max().item())
# bf16 sensitivity: round p to bf16 in float64 chain
s = ref["s"][r:r+1]
srt = s.reshape(8, 64).sort(-1, descending=True).values
print("top-2 logits per head", srt[:, :2].tolist())
