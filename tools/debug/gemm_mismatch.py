"""Where does a bf16-out nr_gemm differ from float64 (rows / cols pattern)?"""
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from news_recommendation_project_v2_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
for (M, N, K) in [(600, 512, 192), (512, 512, 192), (1024, 512, 192), (600, 512, 64), (4096, 2048, 256)]:
    g = torch.Generator().manual_seed(11)
    a = (torch.randn(M, K, generator=g) * 0.2).bfloat16()
    w = (torch.randn(N, K, generator=g) * 0.1).bfloat16()
    b = torch.randn(N, generator=g) * 0.1
    ref = (a.double() @ w.double().T + b.double()).numpy()
    for bias in (b, None):
        out = ops.gemm(a.to(dev), w.to(dev), bias.to(dev) if bias is not None else None, out_dtype=torch.bfloat16)
        torch.cuda.synchronize()
        o = out.float().cpu().double().numpy()
        rr = ref if bias is not None else ref - b.double().numpy()[None, :]
        bad = np.abs(o - rr) > 1e-2 + 1e-2 * np.abs(rr)
        rows = np.flatnonzero(bad.any(1))
        cols = np.flatnonzero(bad.any(0))
        print(f"M={M} N={N} K={K} bias={bias is not None}: bad {bad.sum()} / {bad.size}; rows {rows[:8]}..{rows[-4:] if len(rows) else ''} "
              f"({len(rows)}); cols {cols[:8]}..({len(cols)}); row%16 {np.bincount(rows % 16, minlength=16) if len(rows) else ''} "
              f"col%64 {np.bincount(cols % 64, minlength=64)[:16] if len(cols) else ''}", flush=True)
