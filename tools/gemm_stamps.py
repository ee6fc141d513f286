#!/usr/bin/env python3
"""Phase breakdown of the 256x256 bf16 GEMM from per-block s_memrealtime
stamps (100 MHz): prologue (entry -> first K tile landed), K loop, epilogue
issue, store drain, and the per-CU idle time between consecutive blocks.
Needs the diagnostic build (-DNR_GEMM_STAMPS=1) loaded through NR_HIP_LIB:

    NR_HIP_LIB=.../build_ab/libnewsrec_hip_stamps.so python tools/gemm_stamps.py --n 8192 --k 1024 --epi geglu
"""
import argparse
import ctypes
import json
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from news_recommendation_project_v2_amd import _lib, ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=72023)
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--k", type=int, default=1024)
    ap.add_argument("--epi", default="geglu", choices=["none", "relu", "geglu", "gelu", "exp"])
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    lib = _lib.load()
    fn = lib.nr_debug_gemm_stamps
    fn.restype, fn.argtypes = ctypes.c_int, [ctypes.c_void_p]
    a = (torch.randn(args.m, args.k, device=dev) * 0.1).to(torch.bfloat16)
    w = (torch.randn(args.n, args.k, device=dev) * 0.05).to(torch.bfloat16)
    b = torch.randn(args.n, device=dev) * 0.01
    out = torch.empty(args.m, args.n // 2 if args.epi == "geglu" else args.n, device=dev, dtype=torch.bfloat16)
    blocks = ((args.m + 255) // 256) * (args.n // 256)
    st = torch.zeros(blocks * 8, dtype=torch.int64, device=dev)
    for _ in range(5):  # warm (clock, caches), then the stamped launch
        ops.gemm(a, w, b, epilogue=args.epi, out=out)
    assert fn(st.data_ptr()) == 0
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    ops.gemm(a, w, b, epilogue=args.epi, out=out)
    e1.record()
    torch.cuda.synchronize()
    assert fn(None) == 0
    s = st.view(blocks, 8).cpu().numpy()
    t = s[:, :5].astype(np.float64) * 10.0  # ns (100 MHz)
    t0 = t[:, 0].min()
    t -= t0
    hw, xcc = s[:, 5].astype(np.int64), s[:, 6].astype(np.int64)
    cu_key = xcc * 65536 + ((hw >> 8) & 0xFF)  # XCC + {SE, SH, CU} id bits
    ph = {"prologue_us": (t[:, 1] - t[:, 0]) / 1e3, "kloop_us": (t[:, 2] - t[:, 1]) / 1e3,
          "epilogue_issue_us": (t[:, 3] - t[:, 2]) / 1e3, "store_drain_us": (t[:, 4] - t[:, 3]) / 1e3,
          "block_us": (t[:, 4] - t[:, 0]) / 1e3}
    gaps, per_cu = [], []
    for key in np.unique(cu_key):
        idx = np.where(cu_key == key)[0]
        o = idx[np.argsort(t[idx, 0])]
        per_cu.append(len(o))
        if len(o) > 1:
            gaps.extend(((t[o[1:], 0] - t[o[:-1], 4]) / 1e3).tolist())
    span_us = (t[:, 4].max()) / 1e3
    res = {"shape": f"M={args.m} N={args.n} K={args.k} {args.epi}", "blocks": blocks,
           "kernel_ms_event": round(e0.elapsed_time(e1), 4), "stamp_span_us": round(span_us, 1),
           "cus_seen": int(len(per_cu)), "blocks_per_cu_min_max": [int(min(per_cu)), int(max(per_cu))],
           "turnover_gap_us_median": round(float(np.median(gaps)), 3) if gaps else None,
           "turnover_gap_us_p90": round(float(np.percentile(gaps, 90)), 3) if gaps else None,
           "busy_frac": round(float(ph["block_us"].sum() / (len(per_cu) * span_us)), 4)}
    for k, v in ph.items():
        res[k] = {"median": round(float(np.median(v)), 3), "p10": round(float(np.percentile(v, 10)), 3),
                  "p90": round(float(np.percentile(v, 90)), 3)}
    first = t[:, 0] < 1000.0  # blocks of the first round (started within 1 us)
    res["first_round_prologue_us_median"] = round(float(np.median(ph["prologue_us"][first])), 3)
    res["later_prologue_us_median"] = round(float(np.median(ph["prologue_us"][~first])), 3)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
