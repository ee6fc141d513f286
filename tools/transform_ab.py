#!/usr/bin/env python3
"""A/B (tool only): the bf16 per-news transforms (latent, LN-folded, and
FinalAttention) of two libnewsrec builds, interleaved in one process, each
library called through ctypes with its own workspace size.

    python tools/transform_ab.py --libs new=path head=path [--m 72023 9003]
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
from news_recommendation_project_v2_amd import weights as W  # noqa: E402
from news_recommendation_project_v2_amd.latent_attention import LatentAttentionModel  # noqa: E402
from news_recommendation_project_v2_amd.modeling_utils import FinalAttention  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", nargs="+", required=True)
    ap.add_argument("--m", nargs="+", type=int, default=[72023, 9003])
    ap.add_argument("--rounds", type=int, default=6)
    args = ap.parse_args()
    libs = {kv.split("=", 1)[0]: ctypes.CDLL(kv.split("=", 1)[1]) for kv in args.libs}
    for lib in libs.values():
        lib.nr_latent_workspace_bytes.restype = ctypes.c_int64
        lib.nr_latent_workspace_bytes.argtypes = [ctypes.c_int, ctypes.c_int64]
        lib.nr_final_attn_workspace_bytes.restype = ctypes.c_int64
        lib.nr_final_attn_workspace_bytes.argtypes = [ctypes.c_int, ctypes.c_int64]
        lib.nr_last_error.restype = ctypes.c_char_p
    dev = torch.device("cuda:0")
    lm = LatentAttentionModel()
    lm.load_state_dict(W.latent_attention_state_dict(1234))
    lm = lm.to(dev).eval()
    wl = lm.hip_weights(torch.bfloat16)
    fm = FinalAttention(1024, 4096)
    fm.load_state_dict(W.final_attention_state_dict(1234))
    fm = fm.to(dev).eval()
    wf = fm.hip_weights(torch.bfloat16)
    P = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    L = ctypes.c_int64
    for m in args.m:
        g = torch.Generator(device=dev).manual_seed(m)
        e = torch.randn((m, 1024), generator=g, device=dev).to(torch.bfloat16)
        outs, ws, fns = {}, {}, {}
        for lab, lib in libs.items():
            ws[lab] = (torch.empty(lib.nr_latent_workspace_bytes(1, m), dtype=torch.uint8, device=dev),
                       torch.empty(lib.nr_final_attn_workspace_bytes(1, m), dtype=torch.uint8, device=dev))
            outs[lab] = (torch.empty(m, 1024, dtype=torch.bfloat16, device=dev),
                         torch.empty(m, 2048, dtype=torch.bfloat16, device=dev))

            def lat(lib=lib, lab=lab):
                o, w = outs[lab][0], ws[lab][0]
                rc = lib.nr_latent_transform_lnfold(1, L(m), P(e), L(1024), P(wl["Wq_ln"]), P(wl["ucq"]), P(wl["Bt"]),
                                                    P(wl["Wf_ln"]), P(wl["ucf"]), P(wl["W2"]), P(wl["b2"]), P(o), P(w),
                                                    L(w.numel()), s)
                assert rc == 0, lib.nr_last_error()

            def fin(lib=lib, lab=lab):
                o, w = outs[lab][1], ws[lab][1]
                rc = lib.nr_final_attn_transform(1, L(m), P(e), L(1024), P(wf["W1"]), P(wf["b1"]), P(wf["W2"]),
                                                 P(wf["b2"]), P(wf["W3"]), P(wf["b3"]), P(wf["W4"]), P(wf["b4"]),
                                                 P(wf["W5"]), P(o), P(w), L(w.numel()), s)
                assert rc == 0, lib.nr_last_error()
            fns[lab] = (lat, fin)
        for k, name in enumerate(("latent_lnfold", "final")):
            t = {lab: [] for lab in libs}
            for _ in range(args.rounds):
                for lab in libs:
                    f = fns[lab][k]
                    f()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(5):
                        f()
                    e1.record()
                    torch.cuda.synchronize()
                    t[lab].append(e0.elapsed_time(e1) / 5)
            ref = next(iter(libs))
            diff = {lab: float((outs[lab][k].float() - outs[ref][k].float()).abs().max()) for lab in libs}
            print(json.dumps({"m": m, "transform": name, **{f"{lab}_ms": round(float(np.median(v)), 4)
                                                          for lab, v in t.items()}, "maxdiff_vs_first": diff}),
                  flush=True)


if __name__ == "__main__":
    main()
