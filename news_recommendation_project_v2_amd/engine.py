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
from .data_utils import distinct_segments, lengths_to_offsets

# below this share of impressions that repeat an earlier impression's history,
# the fused pass (which re-gathers a shared history per impression) moves fewer
# bytes than pooling the distinct histories into f32 user rows (+4 KiB written
# and +4 KiB read per user row): break-even ~ 2 x 4 KiB / (33 x 2 KiB) ~ 0.12
DEDUPE_MIN_SHARE = 0.15


def _may_repeat(hist_idx: np.ndarray, hist_len: np.ndarray) -> bool:
    """Cheap bound before the exact grouping: repeated histories share (length,
    first id, last id), so if fewer than DEDUPE_MIN_SHARE of the impressions
    repeat such a triple, fewer repeat a whole history."""
    off = lengths_to_offsets(hist_len)
    nz = hist_len > 0
    first = np.where(nz, hist_idx[np.minimum(off[:-1], max(len(hist_idx) - 1, 0))] if len(hist_idx) else 0, -1)
    last = np.where(nz, hist_idx[np.maximum(off[1:] - 1, 0)] if len(hist_idx) else 0, -1)
    key = (hist_len.astype(np.int64) << 42) ^ (first.astype(np.int64) + 1 << 21) ^ (last.astype(np.int64) + 1)
    return 1.0 - len(np.unique(key)) / len(hist_len) >= DEDUPE_MIN_SHARE


def _check_segments(idx: np.ndarray, lens: np.ndarray, what: str) -> None:
    """Validate one CSR index set's lengths on the host (I entries): negative
    lengths and a length sum that does not match the index array (the offsets
    would run past it on the device) are refused.  The rows themselves are
    range-checked on the device after the upload (_row_range)."""
    if len(lens) and int(lens.min()) < 0:
        raise ValueError(f"{what} lengths must be >= 0")
    if int(lens.sum()) != len(idx):
        raise ValueError(f"{what} lengths sum to {int(lens.sum())} but {len(idx)} indices were given")


def _row_range(idx: torch.Tensor, what: str) -> int:
    """Largest row of an uploaded index array (-1 if empty); a negative row is
    refused (IndexError, as torch indexing does).  One min/max reduction where
    the array already is (on the device: microseconds for the 26 M MIND-large-dev
    rows that took ~20 ms of host passes) and one small sync."""
    if idx.numel() == 0:
        return -1
    lo, hi = (int(v) for v in torch.aminmax(idx))
    if lo < 0:
        raise IndexError(f"{what} index {lo} is negative (rows are 0-based indices into the news table)")
    return hi


def _upload(x, dev: torch.device, dtype: Optional[torch.dtype] = None) -> torch.Tensor:
    """Host arrays / CPU tensors to the device; a table converts to the compute
    dtype on the device.  torch's own host-to-device copy of pageable memory runs
    at the PCIe DMA rate here (56 GB/s for the MIND-large-dev index arrays,
    tools/pcie_probe.py, profiles/round6/pcie_probe.jsonl), faster than staging
    through a ring of pinned chunks (45 GB/s, measured and removed in round 6):
    the round-5 "14 GB/s" upload was load_impressions' host-side checks and
    offsets, not the copy."""
    t = torch.as_tensor(x)
    t = t.to(dev)
    return (t if dtype is None or t.dtype == dtype else t.to(dtype)).contiguous()


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
        self._users = None  # f32 [distinct histories, D], reused across steps

    # ------------------------------------------------------------ inputs
    def load_news(self, news_embeddings: torch.Tensor, query_news_embeddings: Optional[torch.Tensor] = None):
        """Upload the news table (and optional separate history-side table)."""
        self.cand_table = _upload(news_embeddings, self.device, self.dtype)
        if query_news_embeddings is not None:
            self.hist_src = _upload(query_news_embeddings, self.device, self.dtype)
        else:
            self.hist_src = self.cand_table
        self._check_rows()
        return self

    def load_impressions(self, hist_idx, hist_len, cand_idx, cand_len, dedupe: Optional[bool] = None):
        """Upload the CSR index arrays.  ``dedupe`` (default: automatic) pools
        each DISTINCT history once (MIND repeats a user's history on every
        impression of that user) and scores the candidates against the stored
        user rows: same scores bit for bit, fewer gathered bytes once at least
        DEDUPE_MIN_SHARE of the impressions repeat a history."""
        dev = self.device
        if len(hist_len) != len(cand_len):
            raise ValueError("Number of rows should be consistent")  # data_model_helper.py:183-185
        hist_idx = np.ascontiguousarray(hist_idx, dtype=np.int32)
        hist_len = np.asarray(hist_len, dtype=np.int64)
        cand_idx = np.ascontiguousarray(cand_idx, dtype=np.int32)
        cand_len_a = np.asarray(cand_len, dtype=np.int64)
        _check_segments(hist_idx, hist_len, "history")
        _check_segments(cand_idx, cand_len_a, "candidate")
        hi_d, ci_d = _upload(hist_idx, dev), _upload(cand_idx, dev)
        # the kernels index tables with these rows: an out-of-range row would be an
        # out-of-bounds device read, so refuse it here, before the engine takes the
        # arrays (a refused load leaves the previous impressions in place), as torch
        # indexing does (IndexError)
        max_row = {"hist": _row_range(hi_d, "history"), "cand": _row_range(ci_d, "candidate")}
        prev, self._max_row = getattr(self, "_max_row", None), max_row
        try:
            self._check_rows()
        except IndexError:
            self._max_row = prev
            raise
        self.hist_idx, self.cand_idx = hi_d, ci_d
        self.hist_off = _upload(lengths_to_offsets(hist_len), dev)
        self.cand_off = _upload(lengths_to_offsets(cand_len_a), dev)
        self.n_cand = int(cand_len_a.sum())
        self.n_imp = len(cand_len)
        self.user_idx = None
        self.shared_history_share = 0.0
        if dedupe is not False and self.n_imp and (dedupe or _may_repeat(hist_idx, hist_len)):
            group, first = distinct_segments(hist_idx, hist_len)
            self.shared_history_share = 1.0 - len(first) / self.n_imp
            if dedupe or self.shared_history_share >= DEDUPE_MIN_SHARE:
                ho, ulen = lengths_to_offsets(hist_len), hist_len[first]
                uoff = lengths_to_offsets(ulen)
                rows = np.repeat(ho[:-1][first], ulen) + (np.arange(int(uoff[-1])) - np.repeat(uoff[:-1], ulen))
                self.uhist_idx = _upload(hist_idx[rows], dev)
                self.uhist_off = _upload(uoff, dev)
                self.user_idx = _upload(group.astype(np.int32), dev)
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

    def _check_rows(self) -> None:
        """Host-side: every index row of the loaded impressions exists in the loaded
        tables (no device sync; the maxima were taken at load_impressions)."""
        mr = getattr(self, "_max_row", None)
        if mr is None:
            return
        for name, table in (("hist", self.hist_src), ("cand", self.cand_table)):
            if table is not None and mr[name] >= table.shape[0]:
                raise IndexError(f"{'history' if name == 'hist' else 'candidate'} index {mr[name]} is out of bounds "
                                 f"for dimension 0 with size {table.shape[0]}")

    def pool_score(self, want_users: bool = False, scores: Optional[torch.Tensor] = None):
        if self.user_idx is not None:  # distinct histories pooled once, then scored per impression
            n_u = self.uhist_off.numel() - 1
            if self._users is None or self._users.shape[0] != n_u:
                self._users = torch.empty((n_u, 1024), dtype=torch.float32, device=self.device)
            users = ops.pool_users(self.pooler, self.hist_table, self.uhist_idx, self.uhist_off, out=self._users)
            s = ops.score_users(users, self.user_idx, self.cand_table, self.cand_inv, self.cand_idx, self.cand_off,
                                self.n_cand, scores=scores)
            return s, (users[self.user_idx.long()] if want_users else None)
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
