#!/usr/bin/env python3
"""Per-tile phase cycles of the persistent GEMM from the stamped diagnostic
build (tools/gemm_lab/make_stamped.py).  Tool only."""
import ctypes
import json
import sys
from pathlib import Path

import torch

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent))
from gemm_ab import EPI, SHAPES, load, run  # noqa: E402


def main():
    lib = load(HERE / (sys.argv[1] if len(sys.argv) > 1 else "libnewsrec_stamped.so"))
    lib.lab_set_stamps.argtypes = [ctypes.c_void_p]
    dev = torch.device("cuda:0")
    buf = torch.zeros(256 * 8, dtype=torch.int64, device=dev)
    assert lib.lab_set_stamps(ctypes.c_void_p(buf.data_ptr())) == 0
    g = torch.Generator(device=dev).manual_seed(0)
    M = 72023
    for name, n, k, epi in SHAPES:
        a = (torch.rand(M, k, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(n, k, device=dev, generator=g) * 2 - 1) / k ** 0.5).to(torch.bfloat16)
        b = (torch.rand(n, device=dev, generator=g) - 0.5) * 0.1
        nc = n // 2 if epi == "geglu" else n
        r = (torch.rand(M, nc, device=dev, generator=g) - 0.5).to(torch.bfloat16) if epi == "resadd" else None
        out = torch.empty(M, nc, device=dev, dtype=torch.bfloat16)
        for _ in range(3):
            run(lib, a, w, b, epi, r, out)
        torch.cuda.synchronize()
        buf.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        run(lib, a, w, b, epi, r, out)
        e1.record()
        torch.cuda.synchronize()
        s = buf.view(256, 8).double().cpu()
        act = s[:, 4] > 0
        s = s[act]
        tiles = s[:, 4]
        per = {ph: float((s[:, i] / tiles).mean()) for i, ph in enumerate(["main", "pre", "epi", "top"])}
        clock = float((s[:, 5] / s[:, 6]).median() * 100e6)
        res = {"shape": name, "kernel_ms": round(e0.elapsed_time(e1), 4), "tiles_per_block": float(tiles.mean()),
               "clock_GHz": round(clock / 1e9, 3),
               **{f"{ph}_cyc": round(v) for ph, v in per.items()},
               **{f"{ph}_us": round(v / clock * 1e6, 3) for ph, v in per.items()},
               "main_per_ktile_us": round(per["main"] / clock * 1e6 / (k / 64), 4),
               "block_total_us": round(float((s[:, 5] / clock).mean()) * 1e6, 1)}
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
