"""Device-resident eval engine for the embed -> pool -> score hot path.

Layout in HBM (one GPU):
  cand_table  [N, 1024] news embeddings in the compute dtype (f32 | bf16)
  cand_inv    [N] f32   1 / max(||row||, 1e-8)           (cosine clamp)
  hist_table  FinalAttention: [N, 2, 1024] = (x, exp(w)) rows, 4/8 KiB
              Latent        : [N, 1024] per-item hiddens
  hist_idx/hist_off, cand_idx/cand_off   int32 rows + int64 CSR offsets
  scores      [C] f32, ranks [C] int32, users [I, 1024] f32 (optional)

One ``step`` = the per-news pooler transform over all N news (MFMA GEMM
chain), the candidate inverse norms, and the fused pool+score kernel over all
impressions.  Everything is enqueued on the current stream; nothing syncs.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from . import ops
from .data_utils import lengths_to_offsets


class PoolScoreEngine:
    def __init__(self, model: torch.nn.Module, dtype: torch.dtype = torch.float32,
                 device: Optional[torch.device] = None):
        self.model = model
        self.pooler = model.pooler_kind
        self.dtype = dtype
        self.device = device or next(model.parameters()).device
        self.weights = model.hip_weights(dtype)  # prepared once
        self.cand_table = None
        self.hist_src = None
        self.cand_inv = None
        self.hist_table = None
        self._ws = None

    # ------------------------------------------------------------ inputs
    def load_news(self, news_embeddings: torch.Tensor, query_news_embeddings: Optional[torch.Tensor] = None):
        """Upload the news table (and optional separate history-side table)."""
        self.cand_table = news_embeddings.to(self.device, self.dtype).contiguous()
        if query_news_embeddings is not None:
            self.hist_src = query_news_embeddings.to(self.device, self.dtype).contiguous()
        else:
            self.hist_src = self.cand_table
        return self

    def load_impressions(self, hist_idx, hist_len, cand_idx, cand_len):
        dev = self.device
        self.hist_idx = torch.as_tensor(np.ascontiguousarray(hist_idx, dtype=np.int32)).to(dev)
        self.hist_off = torch.as_tensor(lengths_to_offsets(hist_len)).to(dev)
        self.cand_idx = torch.as_tensor(np.ascontiguousarray(cand_idx, dtype=np.int32)).to(dev)
        self.cand_off = torch.as_tensor(lengths_to_offsets(cand_len)).to(dev)
        self.n_cand = int(np.asarray(cand_len, dtype=np.int64).sum())
        self.n_imp = len(cand_len)
        if len(hist_len) != len(cand_len):
            raise ValueError("Number of rows should be consistent")  # data_model_helper.py:183-185
        return self

    # ------------------------------------------------------------ stages
    def _workspace(self, n: int) -> torch.Tensor:
        from . import _lib
        dt = _lib.NR_F32 if self.dtype == torch.float32 else _lib.NR_BF16
        fn = (_lib.load().nr_final_attn_workspace_bytes if self.pooler == "final"
              else _lib.load().nr_latent_workspace_bytes)
        need = fn(dt, n)
        if self._ws is None or self._ws.numel() < need:
            self._ws = torch.empty(need, dtype=torch.uint8, device=self.device)
        return self._ws

    def transform(self, rows: Optional[slice] = None, out: Optional[torch.Tensor] = None,
                  src: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Per-news pooler table for src[rows] (default: all rows of hist_src)."""
        src = self.hist_src if src is None else src
        src = src if rows is None else src[rows]
        ws = self._workspace(src.shape[0])
        if self.pooler == "final":
            return ops.final_attn_transform(src, self.weights, out=out, workspace=ws)
        return ops.latent_transform(src, self.weights, out=out, workspace=ws)

    def inv_norms(self) -> torch.Tensor:
        self.cand_inv = ops.row_inv_norm(self.cand_table, 1e-8, out=self.cand_inv)
        return self.cand_inv

    def pool_score(self, want_users: bool = False, scores: Optional[torch.Tensor] = None):
        return ops.pool_score(self.pooler, self.hist_table, self.cand_table, self.cand_inv, self.hist_idx,
                              self.hist_off, self.cand_idx, self.cand_off, self.n_cand, want_users=want_users,
                              scores=scores)

    def step(self, want_users: bool = False, scores: Optional[torch.Tensor] = None):
        """Full eval pass: transform + inverse norms + pool/score."""
        self.hist_table = self.transform(out=self.hist_table)
        self.inv_norms()
        return self.pool_score(want_users=want_users, scores=scores)

    def rank(self, scores: torch.Tensor) -> torch.Tensor:
        return ops.dense_rank(scores, self.cand_off)
