#!/usr/bin/env python3
"""f32 -> bf16 transpose rate: the 16-B-store kernel (rows % 8 == 0) against the
generic 2-B-store kernel (one row fewer, so the fast path's shape check fails),
HIP events over back-to-back launches.  Prints one JSON line per shape."""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from news_recommendation_project_v2_amd import ops  # noqa: E402


def time_ms(x, reps=50):
    out = torch.empty((x.shape[1], x.shape[0]), dtype=torch.bfloat16, device=x.device)
    for _ in range(5):
        ops.transpose(x, out=out)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        ops.transpose(x, out=out)
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


for rows, cols in [(8320, 1024), (8320, 4096), (8320, 8192), (72023, 1024)]:
    x = torch.randn(rows, cols, device="cuda")
    fast = time_ms(x)
    gen = time_ms(x[:-1])
    nbytes = rows * cols * 6  # f32 read + bf16 write
    print(json.dumps({"rows": rows, "cols": cols, "fast_ms": round(fast, 4), "generic_ms": round(gen, 4),
                      "fast_TBs": round(nbytes / fast / 1e9, 2), "generic_TBs": round(nbytes / gen / 1e9, 2)}),
          flush=True)
