#!/usr/bin/env python3
"""Row-kernel bandwidth at MIND-large shape: LayerNorm (bf16/f32), inverse norms,
HIP-event timed; bytes = read + write of the rows."""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from news_recommendation_project_v2_amd import ops  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    dev = torch.device("cuda:0")
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 72023
    for dt in (torch.bfloat16, torch.float32):
        x = torch.randn(n, 1024, device=dev).to(dt)
        y = torch.empty_like(x)
        g = torch.rand(1024, device=dev) + 0.5
        b = torch.randn(1024, device=dev)
        ms = timeit(lambda: ops.layernorm(x, g, b, 1e-5, out=y))
        byt = 2 * x.numel() * x.element_size()
        ms_t = timeit(lambda: torch.nn.functional.layer_norm(x, (1024,), g.to(dt), b.to(dt), 1e-5))
        print(json.dumps({"kernel": "layernorm", "dtype": str(dt), "rows": n, "ms": round(ms, 4),
                          "GBs": round(byt / ms / 1e6, 1), "torch_ms": round(ms_t, 4)}), flush=True)
        inv = torch.empty(n, device=dev)
        ms = timeit(lambda: ops.row_inv_norm(x, out=inv))
        print(json.dumps({"kernel": "inv_norm", "dtype": str(dt), "ms": round(ms, 4),
                          "GBs": round(x.numel() * x.element_size() / ms / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
