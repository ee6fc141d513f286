#!/usr/bin/env python3
"""Run one GEMM shape a few times (for rocprofv3 --pmc passes).
    python tools/profile_gemm.py N K [epilogue] [M]"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from news_recommendation_project_v2_amd import ops  # noqa: E402

n, k = int(sys.argv[1]), int(sys.argv[2])
epi = sys.argv[3] if len(sys.argv) > 3 else "none"
m = int(sys.argv[4]) if len(sys.argv) > 4 else 72023
reps = int(sys.argv[5]) if len(sys.argv) > 5 else 3
dev = torch.device("cuda:0")
a = (torch.randn(m, k, device=dev) * 0.1).bfloat16()
w = (torch.randn(n, k, device=dev) * 0.05).bfloat16()
b = torch.randn(n, device=dev) * 0.01
out = torch.empty(m, n // 2 if epi == "geglu" else n, device=dev, dtype=torch.bfloat16)
r = torch.randn(m, n, device=dev).bfloat16() if epi == "resadd" else None
for _ in range(reps):
    ops.gemm(a, w, b, epilogue=epi, residual=r, out=out)
torch.cuda.synchronize()
