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


WARM_S = 2.0


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
        # >= 2 s of back-to-back launches on random data first (MI355X_MICROARCH.md
        # "DVFS give-back" item 6): the clock the chip holds under this load
        import time
        t_end = time.perf_counter() + WARM_S
        while time.perf_counter() < t_end:
            for _ in range(20):
                run(lib, a, w, b, epi, r, out)
            torch.cuda.synchronize()
        buf.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        run(lib, a, w, b, epi, r, out)
        e1.record()
        torch.cuda.synchronize()
        s = buf.view(256, 8).double().cpu()
        s = s[s[:, 6] > 0]
        clk = s[:, 5] / s[:, 6] * 100e6  # shader cycles / 100 MHz ticks, per workgroup
        ms = e0.elapsed_time(e1)
        flop = 2.0 * M * (n // 2 if epi == "geglu" else n) * k * (2 if epi == "geglu" else 1)
        res = {"shape": name, "kernel_ms": round(ms, 4), "tflops": round(flop / ms / 1e9, 1),
               "units_per_block": float(s[:, 4].mean()), "workgroups": int(s.shape[0]),
               "clock_GHz_median": round(float(clk.median()) / 1e9, 3),
               "clock_GHz_min": round(float(clk.min()) / 1e9, 3), "clock_GHz_max": round(float(clk.max()) / 1e9, 3),
               "peak_at_clock_TF": round(2500.0 * float(clk.median()) / 2.4e9, 1),
               "warm_s": WARM_S}
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
