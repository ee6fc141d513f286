#!/usr/bin/env python3
"""Same-process A/B of the title-encoder attention kernel: the shipped library
against lab builds (--lab name=path; default tools/attn_lab/libnewsrec_attn2d.so,
the previous 2-D grid: query block x head group, round-robin over the XCDs).

Synthetic packed titles (lengths ~ N(mean, 6), clipped to [4, 512]), random
bf16 qkv [T, 3072]; both libraries run on the same buffers, interleaved, timed
with HIP events on the stream they launch on, back to back (one sync at the end).  Outputs of the two must agree bit
for bit (same per-wave arithmetic, only the dispatch order differs).

    python tools/attn_ab.py --tokens 1000000 --mean-len 20 66 200

The lab library (not shipped; .gpurunignore lists tools/attn_lab) is the shipped
objects relinked with commit 4d743f8~1's encoder.hip:
    git show 4d743f8~1:news_recommendation_project_v2_amd/csrc/encoder.hip > /tmp/enc_old.hip
    (cd news_recommendation_project_v2_amd/csrc && hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I. \
        -c /tmp/enc_old.hip -o /tmp/enc_old.o && hipcc --offload-arch=gfx950 -shared -fPIC \
        build/{capi,gemm,pool_score,rowops,rank}.o /tmp/enc_old.o build/{train,metrics}.o \
        -o ../../tools/attn_lab/libnewsrec_attn2d.so)
Recorded: profiles/round3/s6/attn_ab.jsonl.
"""
import argparse
import ctypes
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from news_recommendation_project_v2_amd import _lib  # noqa: E402

NR_BF16 = 1


def open_lib(path):
    lib = ctypes.CDLL(str(path))
    fn = lib.nr_attention_varlen
    fn.restype = ctypes.c_int
    fn.argtypes = _lib.SIGNATURES["nr_attention_varlen"][1]
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=1_000_000)
    ap.add_argument("--mean-len", type=float, nargs="+", default=[20.0, 66.0, 200.0])
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--lab", nargs="+", default=["rr_2d=tools/attn_lab/libnewsrec_attn2d.so"],
                    help="name=path of lab libraries timed against the shipped one")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    libs = {"shipped": _lib.load()}
    for spec in args.lab:
        name, path = spec.split("=", 1)
        libs[name] = open_lib(ROOT / path)
    stream = torch.cuda.current_stream(dev)
    sp = ctypes.c_void_p(stream.cuda_stream)
    rng = np.random.default_rng(0)
    for mean in args.mean_len:
        lens = []
        while sum(lens) < args.tokens:
            lens.append(int(np.clip(round(rng.normal(mean, 6)), 4, 512)))
        lens = np.array(lens, dtype=np.int64)
        T, n = int(lens.sum()), len(lens)
        qb = np.concatenate([[0], np.cumsum((lens + 31) // 32)]).astype(np.int32)
        cu = torch.tensor(np.concatenate([[0], np.cumsum(lens)]).astype(np.int32), device=dev)
        qo = torch.tensor(qb, device=dev)
        qkv = torch.randn(T, 3072, device=dev).to(torch.bfloat16)
        outs = {k: torch.empty(T, 1024, dtype=torch.bfloat16, device=dev) for k in libs}

        def run(k):
            rc = libs[k].nr_attention_varlen(NR_BF16, n, int(qb[-1]), qkv.data_ptr(), cu.data_ptr(), qo.data_ptr(),
                                             outs[k].data_ptr(), sp)
            assert rc == 0, (k, rc)

        for _ in range(5):  # warm-up (clocks up: the timed launches then run back to back)
            for k in libs:
                run(k)
        ev = {k: [] for k in libs}
        for _ in range(args.reps):
            for k in libs:
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(stream)
                run(k)
                b.record(stream)
                ev[k].append((a, b))
        torch.cuda.synchronize(dev)
        times = {k: [a.elapsed_time(b) for a, b in v] for k, v in ev.items()}
        alg = T * (3072 + 1024) * 2  # q, k, v read once + ctx written, bf16
        res = {"mean_len": mean, "tokens": T, "titles": n, "algorithmic_bytes": alg}
        for k, v in times.items():
            ms = float(np.median(v))
            res[k] = {"median_ms": round(ms, 4), "GBs": round(alg / ms / 1e6, 1)}
            if k != "shipped":  # time of the lab build / time of the shipped one
                res[k]["time_vs_shipped"] = round(ms / res["shipped"]["median_ms"], 3)
                res[k]["bit_identical"] = bool(torch.equal(outs[k], outs["shipped"]))
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
