#!/usr/bin/env python3
"""A/B timing of nr_gemm builds on the pooler-transform shapes (M = MIND-large
news count), interleaved in ONE process (guide §5.4 rule 24), with
torch.matmul (hipBLASLt) beside them as the yardstick, plus a correctness
check of every build against a float64 reference on sampled rows.

    python tools/gemm_ab.py [--m 72023] [--libs name=path ...] [--rounds 5]

A library given as name=path:notail runs with its half-tile tail switched off
(nr_set_gemm_half_tail(0) around each call), so one build can be A/B'd
against itself.

Tool only: each library is loaded with ctypes straight from its path (the
product loader, news_recommendation_project_v2_amd/_lib.py, always loads the
in-tree libnewsrec_hip.so).
"""
import argparse
import ctypes
import json
import sys
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))

EPI = {"none": 0, "relu": 1, "exp": 2, "geglu": 3, "resadd": 4, "gelu": 5, "softmax64": 8}
SHAPES = [  # (name, N, K, epilogue)
    ("final.l1 1024->4096 relu", 4096, 1024, "relu"),
    ("final.l2 4096->4096 relu", 4096, 4096, "relu"),
    ("final.l3 4096->1024", 1024, 4096, "none"),
    ("final.l5 4096->1024 exp", 1024, 4096, "exp"),
    ("latent.S 1024->512 softmax64", 512, 1024, "softmax64"),
    ("latent.B 512->1024 resadd", 1024, 512, "resadd"),
    ("latent.ff1 1024->8192 geglu", 8192, 1024, "geglu"),
    ("latent.ff2 4096->1024 resadd", 1024, 4096, "resadd"),
    # epilogue-cost probes: the ff1 shape without GEGLU, and with a plain GELU
    ("probe.ff1shape 1024->8192 none", 8192, 1024, "none"),
    ("probe.ff1shape 1024->8192 gelu", 8192, 1024, "gelu"),
]


def load(path):
    lib = ctypes.CDLL(str(path))
    _p, _i, _l = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
    lib.nr_gemm.restype = _i
    lib.nr_gemm.argtypes = [_i, _i, _i, _l, _l, _l, _p, _l, _p, _l, _p, _p, _l, _p, _l, _p]
    lib.nr_last_error.restype = ctypes.c_char_p
    return lib


def run(lib, a, w, b, epi, r, out, tail=True):
    if not tail:
        lib.nr_set_gemm_half_tail(0)
    try:
        _run(lib, a, w, b, epi, r, out)
    finally:
        if not tail:
            lib.nr_set_gemm_half_tail(1)


def _run(lib, a, w, b, epi, r, out):
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    p = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None
    rc = lib.nr_gemm(1, 1, EPI[epi], a.shape[0], w.shape[0], a.shape[1], p(a), a.shape[1], p(w), w.shape[1], p(b),
                     p(r), r.shape[1] if r is not None else 0, p(out), out.shape[1], s)
    if rc != 0:
        raise RuntimeError(lib.nr_last_error().decode())


def reference_rows(a, w, b, epi, r, rows):
    x = a[rows].double() @ w.double().T + b.double()
    if epi == "relu":
        return torch.relu(x)
    if epi == "exp":
        return torch.exp(x)
    if epi == "resadd":
        return x + r[rows].double()
    if epi == "softmax64":
        return torch.softmax(x.reshape(len(rows), -1, 64), -1).reshape(len(rows), -1)
    if epi == "gelu":
        return torch.nn.functional.gelu(x)
    if epi == "geglu":
        n = x.shape[1]
        xa = x.reshape(len(rows), n // 64, 2, 32)  # 32-row interleave: (a block, g block) per 64 columns
        return (xa[:, :, 0] * torch.nn.functional.gelu(xa[:, :, 1])).reshape(len(rows), n // 2)
    return x


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=72023)
    ap.add_argument("--libs", nargs="*", default=[f"new={REPO / 'news_recommendation_project_v2_amd' / 'libnewsrec_hip.so'}",
                                                   f"base={REPO / 'tools' / 'gemm_lab' / 'libnewsrec_base.so'}"])
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--shapes", default="")
    args = ap.parse_args()
    libs, tails = {}, {}
    for kv in args.libs:
        lab, path = kv.split("=", 1)
        tails[lab] = not path.endswith(":notail")
        libs[lab] = load(path[:-len(":notail")] if path.endswith(":notail") else path)
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    summary = []
    for name, n, k, epi in SHAPES:
        if args.shapes and not any(s in name for s in args.shapes.split(",")):
            continue
        a = (torch.rand(args.m, k, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(n, k, device=dev, generator=g) * 2 - 1) / k ** 0.5).to(torch.bfloat16)
        b = (torch.rand(n, device=dev, generator=g) - 0.5) * 0.1
        nc = n // 2 if epi == "geglu" else n
        r = (torch.rand(args.m, nc, device=dev, generator=g) - 0.5).to(torch.bfloat16) if epi == "resadd" else None
        outs = {lab: torch.empty(args.m, nc, device=dev, dtype=torch.bfloat16) for lab in libs}
        rows = torch.tensor(sorted(set(np.random.default_rng(1).integers(0, args.m, 64).tolist()) | {args.m - 1}),
                            device=dev)
        ref = reference_rows(a, w, b, epi, r, rows)
        err, first = {}, {}
        for lab, lib in libs.items():
            run(lib, a, w, b, epi, r, outs[lab], tails[lab])
            torch.cuda.synchronize()
            err[lab] = float((outs[lab][rows].double() - ref).abs().max())
            first[lab] = outs[lab].clone()
        fns = {lab: (lambda lib=lib, o=outs[lab], tl=tails[lab]: run(lib, a, w, b, epi, r, o, tl))
               for lab, lib in libs.items()}
        fns["torch"] = lambda: torch.matmul(a, w.T)
        # the same op as a hipBLASLt user runs it: addmm (bias in the GEMM) + torch's epilogue kernels
        b16 = b.to(torch.bfloat16)
        wt = w.T
        if epi == "relu":
            fns["torch_epi"] = lambda: torch.relu_(torch.addmm(b16, a, wt))
        elif epi == "exp":
            fns["torch_epi"] = lambda: torch.exp_(torch.addmm(b16, a, wt))
        elif epi == "resadd":
            fns["torch_epi"] = lambda: torch.addmm(b16, a, wt).add_(r)
        elif epi == "softmax64":
            fns["torch_epi"] = lambda: torch.softmax(torch.addmm(b16, a, wt).view(args.m, -1, 64), -1)
        elif epi == "geglu":
            def _geglu():
                x = torch.addmm(b16, a, wt)
                xa, xg = x.chunk(2, dim=-1)
                return xa * torch.nn.functional.gelu(xg)
            fns["torch_epi"] = _geglu
        else:
            fns["torch_epi"] = lambda: torch.addmm(b16, a, wt)
        times = {lab: [] for lab in fns}
        for _ in range(args.rounds):
            for lab, fn in fns.items():
                for _ in range(2):
                    fn()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.reps):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                times[lab].append(e0.elapsed_time(e1) / args.reps)
        # builds that differ only in scheduling must agree bit for bit, and every
        # timed call (each overwrote outs) with its own first call
        lab0 = next(iter(libs))
        bits = {f"{lab}_bit_equal_{lab0}": bool(torch.equal(first[lab], first[lab0])) for lab in libs}
        bits.update({f"{lab}_repeatable": bool(torch.equal(outs[lab], first[lab])) for lab in libs})
        flop = 2.0 * args.m * n * k
        res = {"shape": name, "M": args.m, "N": n, "K": k,
               **{f"{lab}_ms": round(float(np.median(v)), 4) for lab, v in times.items()},
               **{f"{lab}_tflops": round(flop / (float(np.median(v)) * 1e-3) / 1e12, 1) for lab, v in times.items()},
               **{f"{lab}_maxerr": e for lab, e in err.items()}, **bits}
        print(json.dumps(res), flush=True)
        summary.append(res)
    print(json.dumps({"summary": summary}))


if __name__ == "__main__":
    main()
