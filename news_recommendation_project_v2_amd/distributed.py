"""Multi-GPU eval: one process per GPU, torch.distributed over RCCL (xGMI).

The reference has no distributed code; this is the one
parallel strategy the hot path needs:
  phase A  each rank runs the per-news pooler transform on a contiguous
           1/world slice of the news table (MFMA GEMMs, no communication);
  phase B  ONE all_gather_into_tensor of the [N/world, k*1024] slices
           (RCCL ncclAllGather over xGMI) gives every GPU the full table;
  phase C  impressions are split into contiguous, cost-balanced ranges and
           pooled + scored with no further communication.
Scores stay on their rank; ``gather_scores`` concatenates them in impression
order on rank 0 when the caller wants them on the host.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch
import torch.distributed as dist

from .engine import PoolScoreEngine


def shard_rows(n: int, world: int) -> int:
    """Rows per rank for the news-table shard (ceil), so all shards are equal."""
    return (n + world - 1) // world


def partition_by_cost(hist_len: np.ndarray, cand_len: np.ndarray, world: int, table_row_bytes: int,
                      cand_row_bytes: int) -> np.ndarray:
    """Contiguous impression ranges balanced by the prefix sum of
    cost_i = c_i*(cand_row_bytes + 8) + h_i*(table_row_bytes + 4)  (SURVEY §8(e)).
    Returns ``world + 1`` boundaries."""
    cost = cand_len.astype(np.float64) * (cand_row_bytes + 8) + hist_len.astype(np.float64) * (table_row_bytes + 4)
    cs = np.concatenate([[0.0], np.cumsum(cost)])
    targets = cs[-1] * np.arange(world + 1) / world
    b = np.searchsorted(cs, targets, side="left")
    b[0], b[-1] = 0, len(hist_len)
    return np.maximum.accumulate(b).astype(np.int64)


class ShardedTable:
    """Phase A + B: sharded per-news transform and the one-time all-gather."""

    def __init__(self, engine: PoolScoreEngine, rank: int, world: int, group=None):
        self.eng, self.rank, self.world, self.group = engine, rank, world, group
        n = engine.hist_src.shape[0]
        self.rows = shard_rows(n, world)
        width = 2048 if engine.pooler == "final" else 1024
        if self.rows * world != n:  # pad the source so every rank transforms `rows` rows
            pad = torch.zeros((self.rows * world - n, engine.hist_src.shape[1]), dtype=engine.hist_src.dtype,
                              device=engine.device)
            engine.hist_src = torch.cat([engine.hist_src, pad]).contiguous()
        self.full = torch.empty((self.rows * world, width), dtype=engine.dtype, device=engine.device)
        self.local = self.full[rank * self.rows:(rank + 1) * self.rows] if world == 1 else \
            torch.empty((self.rows, width), dtype=engine.dtype, device=engine.device)

    def build(self) -> torch.Tensor:
        sl = slice(self.rank * self.rows, (self.rank + 1) * self.rows)
        self.eng.transform(rows=sl, out=self.local)
        if self.world > 1:
            dist.all_gather_into_tensor(self.full, self.local, group=self.group)
        self.eng.hist_table = self.full
        return self.full


def sharded_step(table: ShardedTable, want_users: bool = False, scores: Optional[torch.Tensor] = None):
    """One eval pass on this rank: A + B (table), inverse norms, C (pool+score)."""
    table.build()
    table.eng.inv_norms()
    return table.eng.pool_score(want_users=want_users, scores=scores)


def gather_scores(local_scores: torch.Tensor, world: int, group=None) -> Optional[torch.Tensor]:
    """Concatenate per-rank score vectors (impression order) on every rank."""
    if world == 1:
        return local_scores
    n = torch.tensor([local_scores.numel()], device=local_scores.device, dtype=torch.int64)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    m = int(max(int(s) for s in sizes))
    buf = torch.zeros(m, dtype=local_scores.dtype, device=local_scores.device)
    buf[:local_scores.numel()] = local_scores
    outs = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(outs, buf, group=group)
    return torch.cat([o[:int(s)] for o, s in zip(outs, sizes)])
