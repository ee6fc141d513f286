#!/usr/bin/env python3
"""Probe (tool only): can the MFMA-bound per-news transform hide under the
HBM-bound pool_score?  Headline workload (latent, bf16, MIND-large-dev shape).

  1. alone: transform, inv_norm, pool_score, serial step (HIP events)
  2. pool_score / transform on CU-masked streams (hipExtStreamCreateWithCUMask)
     of k CUs, mask bits contiguous vs strided, to see how many CUs each needs
  3. two-deep pipelined steps: step i+1's transform (stream B, double-buffered
     table) beside step i's pool_score (stream A), unmasked and with CU splits

    python tools/overlap_probe.py > gpurun_out/overlap/probe.jsonl
"""
import ctypes
import json
import sys
import time
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))

from news_recommendation_project_v2_amd import ops, synthetic  # noqa: E402
from news_recommendation_project_v2_amd import weights as W  # noqa: E402
from news_recommendation_project_v2_amd.engine import PoolScoreEngine  # noqa: E402
from news_recommendation_project_v2_amd.latent_attention import LatentAttentionModel  # noqa: E402

HIP = ctypes.CDLL("libamdhip64.so")
HIP.hipExtStreamCreateWithCUMask.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32,
                                             ctypes.POINTER(ctypes.c_uint32)]
N_CU = torch.cuda.get_device_properties(0).multi_processor_count


def out(**kw):
    print(json.dumps(kw), flush=True)


def masked_stream(bits):
    words = [0] * ((N_CU + 31) // 32)
    for b in bits:
        words[b // 32] |= 1 << (b % 32)
    arr = (ctypes.c_uint32 * len(words))(*words)
    h = ctypes.c_void_p()
    rc = HIP.hipExtStreamCreateWithCUMask(ctypes.byref(h), len(words), arr)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(h.value)


def ev_time(fn, stream, reps=5):
    with torch.cuda.stream(stream):
        fn()
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    with torch.cuda.stream(stream):
        for _ in range(reps):
            fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    m = LatentAttentionModel()
    m.load_state_dict(W.latent_attention_state_dict(1234))
    m = m.to(dev).eval()
    n_news = 72023
    g = torch.Generator(device=dev).manual_seed(1234)
    table = torch.randn((n_news, 1024), generator=g, device=dev)
    imps = synthetic.mind_impressions(n_news, 376471, seed=1234)
    eng = PoolScoreEngine(m, dtype=torch.bfloat16, device=dev).load_news(table)
    eng.load_impressions(imps.hist_idx, imps.hist_len, imps.cand_idx, imps.cand_len)
    scores = torch.empty(imps.n_cand, dtype=torch.float32, device=dev)
    bufs = [eng.transform(), None]
    bufs[1] = torch.empty_like(bufs[0])
    eng.hist_table = bufs[0]
    eng.inv_norms()
    torch.cuda.synchronize()
    default = torch.cuda.current_stream()

    def tx(b=1):
        eng.transform(out=bufs[b])

    def ps(b=0):
        eng.hist_table = bufs[b]
        eng.pool_score(scores=scores)

    def step():
        tx(0)
        eng.inv_norms()
        ps(0)

    t_tx, t_ps, t_step = ev_time(tx, default), ev_time(ps, default), ev_time(step, default)
    out(probe="alone", n_cu=N_CU, transform_ms=round(t_tx, 4), pool_score_ms=round(t_ps, 4),
        serial_step_ms=round(t_step, 4))

    # two-deep pipeline: transform of step i+1 beside pool_score of step i
    def pipelined(sA, sB, steps=10, gemm_wgs=0):
        ops.set_persistent_workgroups(gemm_wgs)
        ev_tx = [torch.cuda.Event(), torch.cuda.Event()]
        ev_ps = [torch.cuda.Event(), torch.cuda.Event()]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(sB):
            tx(0)
        ev_tx[0].record(sB)
        for i in range(steps):
            b, nb = i % 2, (i + 1) % 2
            if i + 1 < steps:
                if i >= 1:
                    sB.wait_event(ev_ps[nb])
                with torch.cuda.stream(sB):
                    tx(nb)
                ev_tx[nb].record(sB)
            sA.wait_event(ev_tx[b])
            with torch.cuda.stream(sA):
                eng.inv_norms()
                ps(b)
            ev_ps[b].record(sA)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps
        ops.set_persistent_workgroups(0)
        return dt * 1e3

    split = sys.argv[1] if len(sys.argv) > 1 else "none"
    if split.startswith("mchunks"):
        # the transform alone, its rows cut into n chunks on n streams (each
        # chunk's GEMM chain in order; the chunks' tail rounds may overlap)
        nch = int(split.split(":")[1])
        streams = [torch.cuda.Stream() for _ in range(nch)]
        bounds = [round(i * n_news / nch) for i in range(nch + 1)]
        from news_recommendation_project_v2_amd import _lib
        wss = [torch.empty(_lib.load().nr_latent_workspace_bytes(_lib.NR_BF16, bounds[i + 1] - bounds[i]),
                           dtype=torch.uint8, device=dev) for i in range(nch)]
        w = eng.weights

        def txc():
            cur = torch.cuda.current_stream()
            ev = torch.cuda.Event()
            ev.record(cur)
            for i, s_ in enumerate(streams):
                s_.wait_event(ev)
                with torch.cuda.stream(s_):
                    ops.latent_transform(eng.cand_table[bounds[i]:bounds[i + 1]], w,
                                         out=bufs[1][bounds[i]:bounds[i + 1]], workspace=wss[i])
            for s_ in streams:
                e2 = torch.cuda.Event()
                e2.record(s_)
                cur.wait_event(e2)

        t1 = ev_time(lambda: tx(1), default, 10)
        tn = ev_time(txc, default, 10)
        torch.cuda.synchronize()
        err = (bufs[1].float() - bufs[0].float()).abs().max().item()
        out(probe="mchunks", chunks=nch, transform_ms=round(t1, 4), chunked_ms=round(tn, 4), max_diff=err)
        return
    if split == "none":
        sA, sB = torch.cuda.Stream(), torch.cuda.Stream()
        kg = 0
    else:
        # "<layout>:<gemm CUs>"; the mask bits are XCD-major (bits 32x..32x+31 = XCD x,
        # measured: contiguous masks of 64/96/128 CUs gather at 2/3/4 XCDs' bandwidth)
        layout, kg = split.split(":")
        kg = int(kg)
        if layout == "xcd":  # whole XCDs for the GEMM (the last kg/32), the rest for pool_score
            gb = list(range(N_CU - kg, N_CU))
        elif layout == "sa":  # pool_score on every (N_CU / (N_CU - kg))-th bit, the GEMM on the rest
            stride = N_CU // (N_CU - kg)
            gb = [i for i in range(N_CU) if i % stride]
        else:  # "cu": kg/8 CUs of every XCD for the GEMM
            per = kg // 8
            gb = [x * (N_CU // 8) + j for x in range(8) for j in range(per)]
        pb = [i for i in range(N_CU) if i not in set(gb)]
        sA, sB = masked_stream(pb), masked_stream(gb)
    ops.set_persistent_workgroups(kg)
    r = {"probe": "split", "split": split, "gemm_cus": kg or N_CU,
         "pool_cus": N_CU - kg if kg else N_CU,
         "transform_alone_ms": round(ev_time(lambda: tx(1), sB), 4)}
    ops.set_persistent_workgroups(0)
    r["pool_score_alone_ms"] = round(ev_time(lambda: ps(0), sA), 4)
    pipelined(sA, sB, 3, kg)
    r["pipelined_ms_per_step"] = round(pipelined(sA, sB, 10, kg), 4)
    r["pipelined_ms_per_step_2"] = round(pipelined(sA, sB, 10, kg), 4)
    out(**r)


if __name__ == "__main__":
    main()
