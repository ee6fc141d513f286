#!/usr/bin/env python3
"""Headline benchmark: scored candidates/sec on MIND-large-shaped impressions.

    python bench.py [--gpus N --steps K --warmup W --pooler latent|final --dtype bf16|fp32]

Workload (BASELINE.json configs[2], "MIND-large eval on 1xMI355X, bf16"):
synthetic MIND-large-dev-shaped impressions (N = 72,023 news, I = 376,471
impressions per GPU, h ~ geometric(1/33), c ~ geometric(1/37)), a seeded
N(0,1) news table resident in HBM, deterministic random-init pooler weights
(no checkpoint exists).  One step = the per-news pooler transform over all N
news (MFMA GEMM chain) + candidate inverse norms + the fused pool+score kernel
over every impression, i.e. everything `scripts/eval.py` computes between
loading the table and ranking.  For N > 1 (one process per GPU under
torch.distributed.run, RCCL) every rank owns its own MIND-large-dev-sized
impression set (weak scaling); the news-table transform is sharded N ways and
all-gathered once per step over xGMI.

Also reported in the same JSON line:
  roofline      the pool+score kernel (dominant, HBM-bound): algorithmic bytes
                per launch / its HIP-event-timed average duration vs 8 TB/s
  cpu_baseline  the oracle (reference algorithm restated on PyTorch CPU:
                padded batches of 128, pooler per padded slot, per-impression
                cosine loop) timed on this host on a bounded sample
  extra         the FinalAttention pooler (the one scripts/eval.py runs), the
                f32 numbers, per-stage times, and the bf16-vs-f32 AUC check
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO))

from news_recommendation_project_v2_amd import synthetic  # noqa: E402
from news_recommendation_project_v2_amd import weights as W  # noqa: E402
from news_recommendation_project_v2_amd.distributed import ShardedTable, sharded_step  # noqa: E402
from news_recommendation_project_v2_amd.engine import PoolScoreEngine  # noqa: E402
from news_recommendation_project_v2_amd.latent_attention import LatentAttentionModel  # noqa: E402
from news_recommendation_project_v2_amd.modeling_utils import FinalAttention  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
MFMA_PEAK_TFLOPS = {"bf16": 2500.0, "fp32": 157.3}
DTYPES = {"bf16": torch.bfloat16, "fp32": torch.float32}


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def make_model(pooler: str, dev):
    if pooler == "final":
        m = FinalAttention(1024, 4096)
        m.load_state_dict(W.final_attention_state_dict(1234))
    else:
        m = LatentAttentionModel()
        m.load_state_dict(W.latent_attention_state_dict(1234))
    return m.to(dev).eval()


def news_table(n: int, dev) -> torch.Tensor:
    g = torch.Generator(device=dev)
    g.manual_seed(1234)
    return torch.randn((n, 1024), generator=g, device=dev, dtype=torch.float32)


def ps_bytes(imps, pooler: str, es: int) -> int:
    """Algorithmic bytes of one pool+score launch (streaming model:
    every gathered row counted once per use)."""
    k = 2 if pooler == "final" else 1
    return (imps.n_cand * (1024 * es + 4 + 4 + 4) + imps.n_hist * (k * 1024 * es + 4) + imps.n_imp * 16)


def tx_flops(n: int, pooler: str) -> float:
    if pooler == "final":
        return n * 2.0 * (1024 * 4096 * 2 + 4096 * 4096 + 4096 * 1024 * 2)
    # folded latent: 1024->512, 512->1024, 1024->8192, 4096->1024
    return n * 2.0 * (1024 * 512 + 512 * 1024 + 1024 * 8192 + 4096 * 1024)


class Run:
    def __init__(self, pooler, dtype, imps, table, dev, rank, world):
        self.pooler, self.dtype = pooler, dtype
        self.model = make_model(pooler, dev)
        self.eng = PoolScoreEngine(self.model, dtype=DTYPES[dtype], device=dev).load_news(table)
        self.eng.load_impressions(imps.hist_idx, imps.hist_len, imps.cand_idx, imps.cand_len)
        self.tab = ShardedTable(self.eng, rank, world)
        self.scores = torch.empty(imps.n_cand, dtype=torch.float32, device=dev)
        self.imps = imps

    def step(self):
        return sharded_step(self.tab, scores=self.scores)

    def stage_times(self, reps: int = 3):
        """HIP-event times (ms) of each stage, events on the launch stream."""
        s = torch.cuda.current_stream()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
        acc = np.zeros(3)
        for _ in range(reps):
            ev[0].record(s)
            self.tab.build()
            ev[1].record(s)
            self.eng.inv_norms()
            ev[2].record(s)
            self.eng.pool_score(scores=self.scores)
            ev[3].record(s)
            torch.cuda.synchronize()
            acc += [ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2]), ev[2].elapsed_time(ev[3])]
        return acc / reps


def timed(run: Run, steps: int, warmup: int, world: int, dev):
    for _ in range(warmup):
        run.step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        run.step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    return dt


def auc_of(run: Run) -> float:
    """Mean AUC over all impressions: dense ranks + per-impression metrics on the
    device (nr_dense_rank, nr_impression_metrics; == evaluation.score, tested)."""
    from news_recommendation_project_v2_amd import evaluation
    s, _ = run.step()
    r = run.eng.rank(s)
    return float(evaluation.score_device(r, run.imps.labels, run.imps.cand_off())["auc"])


def metrics_ms(run: Run, reps: int = 3) -> float:
    """Device time of dense ranks + MIND metrics over the whole workload."""
    from news_recommendation_project_v2_amd import ops
    s, _ = run.step()
    y = torch.as_tensor(np.asarray(run.imps.labels, dtype=np.float32)).to(s.device)
    off = torch.as_tensor(run.imps.cand_off()).to(s.device)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        r = run.eng.rank(s)
        ops.impression_metrics(r, y, off)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def train_step_ms(dev, batch_rows: int = 256, steps: int = 10) -> dict:
    """Config 5 (BASELINE configs[4]): one FinalAttentionTrainStep (fwd + bwd +
    clip + AdamW, bf16 MFMA) on a synthetic MIND-shaped batch."""
    from news_recommendation_project_v2_amd.modeling_utils import get_token_attn_model
    from news_recommendation_project_v2_amd.train_step import FinalAttentionTrainStep, TrainBatch
    rng = np.random.default_rng(1234)
    h = np.clip(rng.geometric(1 / 33.0, batch_rows), 1, 600)
    ids = rng.integers(0, 40_000, int(h.sum()) + 2 * batch_rows)
    uniq, rev = np.unique(ids, return_inverse=True)
    Hs = int(h.sum())
    tok = torch.randn((len(uniq), 1024), generator=torch.Generator().manual_seed(1)).half().to(dev)
    b = TrainBatch(tok, torch.as_tensor(rev[:Hs].astype(np.int32)).to(dev),
                   torch.as_tensor(np.concatenate([[0], np.cumsum(h)]).astype(np.int64)).to(dev),
                   torch.as_tensor(rev[Hs:Hs + batch_rows].astype(np.int32)).to(dev),
                   torch.as_tensor(rev[Hs + batch_rows:].astype(np.int32)).to(dev))
    tm = get_token_attn_model()
    tm.load_state_dict(W.token_attn_state_dict(1234))
    fa = FinalAttention(1024, 4096)
    fa.load_state_dict(W.final_attention_state_dict(1234))
    eng = FinalAttentionTrainStep(tm, fa.to(dev), dtype=torch.bfloat16, device=dev)
    for _ in range(3):
        eng.step(b)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        eng.step(b)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    return {"batch_rows": batch_rows, "history_slots": Hs, "ms_per_step": round(ms, 3),
            "rows_per_s": round(batch_rows / ms * 1e3, 1),
            "gemm_tflops": round(eng.flops_per_step(Hs) / ms / 1e9, 1)}


def cpu_baseline(pooler: str, imps, table_cpu: torch.Tensor, budget_s: float):
    """Reference algorithm (oracle, PyTorch CPU f32) on the first impressions of
    the same workload, batches of 128 until ~budget_s of CPU work."""
    from oracle import pool_ref
    cores = min(16, len(os.sched_getaffinity(0)))
    torch.set_num_threads(cores)
    sd = W.final_attention_state_dict(1234) if pooler == "final" else W.latent_attention_state_dict(1234)
    ho, co = imps.hist_off(), imps.cand_off()
    done_imp, done_cand, t_used, parts = 0, 0, 0.0, []
    while t_used < budget_s and done_imp < imps.n_imp:
        a, b = done_imp, min(done_imp + 128, imps.n_imp)
        t0 = time.perf_counter()
        parts.append(pool_ref.cos_sim_scores(pooler, sd, imps.hist_idx[ho[a]:ho[b]], imps.hist_len[a:b],
                                             imps.cand_idx[co[a]:co[b]], imps.cand_len[a:b], table_cpu))
        t_used += time.perf_counter() - t0
        done_cand += int(co[b] - co[a])
        done_imp = b
    cpu = platform.processor() or platform.machine()
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    res = {"value": done_cand / t_used, "unit": "scored candidates/s", "cores": cores, "kind": "port",
           "sample": f"first {done_imp} impressions ({done_cand} candidates) of the same synthetic workload, "
                     f"{pooler} pooler, f32, {t_used:.1f}s on {cores} threads of {cpu}"}
    return res, done_imp, torch.cat(parts).numpy()


def auc_vs_cpu(runs: dict, imps, n_imp: int, cpu_scores: np.ndarray) -> dict:
    """BASELINE's parity half: mean AUC of the GPU path (device scores -> device
    dense ranks -> device metrics) vs the CPU reference restatement (oracle f32
    scores -> scipy rankdata -> sklearn roc_auc_score per impression), on the
    impressions the CPU leg scored."""
    from news_recommendation_project_v2_amd import evaluation
    from oracle import data_ref, pool_ref
    co = imps.cand_off()
    nc = int(co[n_imp])
    grouped_y = [imps.labels[co[i]:co[i + 1]] for i in range(n_imp)]
    cpu = data_ref.score(pool_ref.dense_ranks(cpu_scores, imps.cand_len[:n_imp]), grouped_y)
    out = {"impressions": n_imp, "candidates": nc, "cpu_ref": {k: cpu[k] for k in ("auc", "mrr", "ndcg5", "ndcg10")}}
    for name, run in runs.items():
        s, _ = run.step()
        r = run.eng.rank(s)[:nc]
        g = evaluation.score_device(r, imps.labels[:nc], co[:n_imp + 1])
        out[name] = {k: g[k] for k in ("auc", "mrr", "ndcg5", "ndcg10")}
        out[name]["max_abs_score_diff"] = float(np.abs(s[:nc].cpu().numpy() - cpu_scores).max())
        out[name]["auc_abs_diff"] = abs(g["auc"] - cpu["auc"])
        out[name]["auc_equal_4dp"] = round(g["auc"], 4) == round(cpu["auc"], 4)
    return out


def load_traffic(pooler: str, dtype: str):
    p = REPO / "profiles" / "pmc_pool_score.json"
    if p.is_file():
        d = json.loads(p.read_text())
        return d.get(f"{pooler}_{dtype}")
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--pooler", choices=["latent", "final"], default="latent")
    ap.add_argument("--dtype", choices=["bf16", "fp32"], default="bf16")
    ap.add_argument("--shape", default="mind_large_dev", choices=list(synthetic.SHAPES))
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-extra", action="store_true", help="headline config only")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: WORLD_SIZE={world} but --gpus={args.gpus}; using WORLD_SIZE")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    n_news, n_imp = synthetic.SHAPES[args.shape]
    t0 = time.time()
    imps = synthetic.mind_impressions(n_news, n_imp, seed=1234 + rank)
    table = news_table(n_news, dev)
    log(f"[bench] data ready in {time.time() - t0:.1f}s: N={n_news} I={imps.n_imp} C={imps.n_cand} H={imps.n_hist}")

    head = Run(args.pooler, args.dtype, imps, table, dev, rank, world)
    dt = timed(head, args.steps, args.warmup, world, dev)
    ms = dt / args.steps * 1e3
    total_cand = imps.n_cand * world  # every rank holds a same-sized set
    if world > 1:
        c = torch.tensor([imps.n_cand], dtype=torch.int64, device=dev)
        dist.all_reduce(c)
        total_cand = int(c.item())
    value = total_cand / (dt / args.steps)
    stages = head.stage_times()
    es = 2 if args.dtype == "bf16" else 4
    bytes_ps = ps_bytes(imps, args.pooler, es)
    achieved = bytes_ps / (stages[2] * 1e-3) / 1e9
    log(f"[bench] {args.pooler}/{args.dtype}: {ms:.2f} ms/step, {value:.3e} cand/s; stages ms "
        f"transform+gather={stages[0]:.2f} invnorm={stages[1]:.3f} pool_score={stages[2]:.2f}")

    extra = {"stage_ms": {"transform_allgather": round(stages[0], 3), "inv_norm": round(stages[1], 4),
                          "pool_score": round(stages[2], 3)},
             "transform_tflops": round(tx_flops(n_news, args.pooler) / world / (stages[0] * 1e-3) / 1e12, 1),
             "transform_peak_frac": round(tx_flops(n_news, args.pooler) / world / (stages[0] * 1e-3) / 1e12
                                          / MFMA_PEAK_TFLOPS[args.dtype], 3),
             "step_roofline_frac": round((bytes_ps / (HBM_PEAK_GBS * 1e9)
                                          + tx_flops(n_news, args.pooler) / world / (MFMA_PEAK_TFLOPS[args.dtype] * 1e12))
                                         / (ms * 1e-3), 4),
             "n_news": n_news, "impressions_per_gpu": imps.n_imp, "candidates_per_gpu": imps.n_cand,
             "history_slots_per_gpu": imps.n_hist}
    if not args.no_extra:
        for pooler, dtype in [(args.pooler, "fp32" if args.dtype == "bf16" else "bf16"),
                              ("final" if args.pooler == "latent" else "latent", args.dtype)]:
            r = Run(pooler, dtype, imps, table, dev, rank, world)
            d = timed(r, max(3, args.steps // 2), 2, world, dev)
            st = r.stage_times(2)
            e2 = 2 if dtype == "bf16" else 4
            extra[f"{pooler}_{dtype}"] = {
                "value": round(total_cand / (d / max(3, args.steps // 2)), 1),
                "ms_per_step": round(d / max(3, args.steps // 2) * 1e3, 3),
                "pool_score_ms": round(st[2], 3), "transform_ms": round(st[0], 3),
                "pool_score_GBs": round(ps_bytes(imps, pooler, e2) / (st[2] * 1e-3) / 1e9, 1)}
            if pooler == args.pooler:
                extra["auc"] = {args.dtype: auc_of(head), dtype: auc_of(r)}
                extra["auc"]["abs_diff"] = abs(extra["auc"][args.dtype] - extra["auc"][dtype])
            del r
            torch.cuda.empty_cache()
        # throughput on the MIND-large *test* shape and cache sensitivity under Zipf(1.1) id popularity
        for tag, shape, zipf in [("mind_large_test", "mind_large_test", None), ("zipf1.1", args.shape, 1.1)]:
            nn_, ni_ = synthetic.SHAPES[shape]
            im = synthetic.mind_impressions(nn_, ni_, seed=1234 + rank, zipf=zipf)
            tb = table if nn_ == n_news else news_table(nn_, dev)
            r = Run(args.pooler, args.dtype, im, tb, dev, rank, world)
            d = timed(r, 3, 1, world, dev) / 3
            st = r.stage_times(2)
            extra[tag] = {"n_news": nn_, "impressions_per_gpu": im.n_imp, "candidates_per_gpu": im.n_cand,
                          "value": round(im.n_cand * world / d, 1), "ms_per_step": round(d * 1e3, 3),
                          "pool_score_ms": round(st[2], 3),
                          "pool_score_GBs": round(ps_bytes(im, args.pooler, es) / (st[2] * 1e-3) / 1e9, 1)}
            del r, tb, im
            torch.cuda.empty_cache()
        extra["metrics_ms"] = round(metrics_ms(head), 3)
        # PCIe-side costs (never part of `value`): the CSR index upload incl. its host-side
        # offsets (load_impressions is idempotent) and the score download
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        head.eng.load_impressions(imps.hist_idx, imps.hist_len, imps.cand_idx, imps.cand_len)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        head.scores.cpu()
        t2 = time.perf_counter()
        extra["pcie_ms"] = {"h2d_index_arrays": round((t1 - t0) * 1e3, 3), "d2h_scores": round((t2 - t1) * 1e3, 3),
                            "index_bytes": int(4 * (imps.n_hist + imps.n_cand) + 8 * 2 * (imps.n_imp + 1)),
                            "score_bytes": int(4 * imps.n_cand)}
        extra["train_bf16_config5"] = train_step_ms(dev)

    cpu = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        log("[bench] timing the CPU reference restatement ...")
        cpu, n_cpu, cpu_scores = cpu_baseline(args.pooler, imps, table.cpu(), args.cpu_seconds)
        runs = {f"gpu_{args.dtype}": head}
        if not args.no_extra:
            runs[f"gpu_{'fp32' if args.dtype == 'bf16' else 'bf16'}"] = Run(
                args.pooler, "fp32" if args.dtype == "bf16" else "bf16", imps, table, dev, rank, world)
        extra["auc_vs_cpu_ref"] = auc_vs_cpu(runs, imps, n_cpu, cpu_scores)
        log(f"[bench] AUC vs CPU reference: {json.dumps(extra['auc_vs_cpu_ref'])}")

    if rank == 0:
        out = {
            "metric": "scored candidates/sec on MIND-large impressions; AUC parity vs CPU ref",
            "value": round(value, 1),
            "unit": "scored candidates/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic (seeded MIND-large-dev-shaped impressions, N(0,1) news table, deterministic "
                    "random-init pooler weights)",
            "config": {"workload": f"{args.shape} eval, {args.pooler} pooler: per-news transform + pool + "
                                   f"cosine score", "pooler": args.pooler, "n_news": n_news,
                       "impressions_per_gpu": imps.n_imp, "parallelism": f"impressions x{world}, news-table "
                                                                         f"transform sharded + all-gather"},
            "roofline": {"bound": "hbm", "kernel": "pool_score_kernel", "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": load_traffic(args.pooler, args.dtype),
                         "algorithmic_bytes_per_launch": bytes_ps, "avg_launch_ms": round(stages[2], 4)},
            "cpu_baseline": cpu,
            "extra": extra,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
