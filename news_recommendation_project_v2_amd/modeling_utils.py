"""Poolers and pooling helpers of the hot path (reference modeling_utils.py).

``FinalAttention`` keeps the reference parameter names (modeling_utils.py:185-192)
so ``load_state_dict`` of a reference checkpoint works unchanged; its forward
runs the MI355X path: the per-item MLP is computed once per valid history row
by the MFMA GEMM chain (``nr_final_attn_transform``) and the per-dimension
softmax pooling by the segmented kernel (``nr_pool_score``).
"""
from __future__ import annotations

from pathlib import Path
from typing import Dict, Optional

import torch
import torch.nn.functional as F

from . import ops
from ._lib import NewsRecHIPError
from .config import DEVICE, FINAL_ATTENTION_HIDDEN_DIM, REDUCED_DIM
from .latent_attention import LatentAttentionModel


def last_token_pool(last_hidden_states: torch.Tensor, attention_mask: torch.Tensor) -> torch.Tensor:
    """Hidden state of each row's last valid token (modeling_utils.py:37-48):
    if every row's last mask slot is set (left padding) take [:, -1], else
    index mask.sum - 1."""
    if bool((attention_mask[:, -1].sum() == attention_mask.shape[0]).item()):
        return last_hidden_states[:, -1]
    last = attention_mask.sum(dim=1) - 1
    return last_hidden_states[torch.arange(last_hidden_states.shape[0], device=last_hidden_states.device), last]


def first_token_pool(last_hidden_states: torch.Tensor, *args, **kwargs) -> torch.Tensor:
    return last_hidden_states[:, 0]


def average_pool(last_hidden_states: torch.Tensor, attention_mask: torch.Tensor) -> torch.Tensor:
    """Masked mean over tokens (modeling_utils.py:55-59)."""
    m = attention_mask[..., None].to(last_hidden_states.dtype)
    return (last_hidden_states * m).sum(dim=1) / attention_mask.sum(dim=1)[..., None]


def flatten_valid(embeddings: torch.Tensor, attention_mask: torch.Tensor):
    """Padded [B, L, D] + mask -> (valid rows [n, D], CSR offsets [B+1] int64).

    The reference feeds zero-padded slots through the pooler and masks them
    out afterwards (data_utils.py:789, modeling_utils.py:224); only valid rows
    matter, so the HIP path never touches the padding.
    """
    mask = attention_mask.to(torch.bool)
    rows = embeddings[mask]
    counts = mask.sum(dim=1).to(torch.int64)
    off = torch.zeros(mask.shape[0] + 1, dtype=torch.int64, device=embeddings.device)
    off[1:] = torch.cumsum(counts, 0)
    return rows.contiguous(), off


def pool_rows(pooler: str, table: torch.Tensor, hist_off: torch.Tensor) -> torch.Tensor:
    """Pool consecutive table rows per segment with the HIP kernel (no candidates)."""
    n = table.shape[0]
    dev = table.device
    hist_idx = torch.arange(n, dtype=torch.int32, device=dev)
    n_seg = hist_off.numel() - 1
    cand_off = torch.zeros(n_seg + 1, dtype=torch.int64, device=dev)
    cand_tab = torch.zeros((1, 1024), dtype=table.dtype, device=dev)
    cand_inv = torch.zeros(1, dtype=torch.float32, device=dev)
    empty = torch.zeros(1, dtype=torch.int32, device=dev)
    _, users = ops.pool_score(pooler, table, cand_tab, cand_inv, hist_idx, hist_off, empty, cand_off, 0,
                              want_users=True)
    return users


class FinalAttention(torch.nn.Module):
    """Additive per-dimension attention pooler (modeling_utils.py:175-228).

    forward(emb [B, L, D], mask [B, L]) -> [B, D]:
      x = W3 relu(W2 relu(W1 e + b1) + b2) + b3 ;  w = W5 relu(W4 x + b4)
      out = sum_L x * exp(w) * m / (sum_L exp(w) * m + 1e-10)
    Dropouts (p=0.1) exist for state/API parity and are inactive in eval.
    """

    def __init__(self, reduced_dim: int, hidden_dim: int):
        super().__init__()
        self.linear1 = torch.nn.Linear(reduced_dim, hidden_dim)
        self.dropout1 = torch.nn.Dropout(0.1)
        self.linear2 = torch.nn.Linear(hidden_dim, hidden_dim)
        self.dropout2 = torch.nn.Dropout(0.1)
        self.linear3 = torch.nn.Linear(hidden_dim, reduced_dim)
        self.linear4 = torch.nn.Linear(reduced_dim, hidden_dim)
        self.dropout3 = torch.nn.Dropout(0.1)
        self.linear5 = torch.nn.Linear(hidden_dim, reduced_dim, bias=False)
        self._hip_cache: Dict[tuple, dict] = {}

    pooler_kind = "final"

    def _param_key(self, dtype):
        ps = list(self.parameters())
        return (dtype, ps[0].device, tuple((p.data_ptr(), p._version) for p in ps))

    def hip_weights(self, dtype: torch.dtype = torch.float32) -> dict:
        """Device weights for nr_final_attn_transform (cached until params change)."""
        key = self._param_key(dtype)
        w = self._hip_cache.get(key)
        if w is None:
            with torch.no_grad():
                w = {}
                for i in range(1, 6):
                    lin = getattr(self, f"linear{i}")
                    w[f"W{i}"] = lin.weight.detach().to(dtype).contiguous()
                    if lin.bias is not None:
                        w[f"b{i}"] = lin.bias.detach().float().contiguous()
            self._hip_cache = {key: w}
        return w

    def item_table(self, rows: torch.Tensor, dtype: Optional[torch.dtype] = None) -> torch.Tensor:
        """Per-item (x, exp(w)) table [n, 2D] for rows [n, D] (one per unique news)."""
        dtype = dtype or rows.dtype
        return ops.final_attn_transform(rows.to(dtype).contiguous(), self.hip_weights(dtype))

    def forward(self, embeddings: torch.Tensor, attention_mask: torch.Tensor) -> torch.Tensor:
        if embeddings.device.type != "cuda":
            raise NewsRecHIPError("FinalAttention.forward runs on the MI355X HIP path only (got a CPU tensor)")
        if self.training:
            raise NewsRecHIPError("FinalAttention HIP forward is inference-only (dropout inactive); call .eval()")
        rows, off = flatten_valid(embeddings, attention_mask)
        table = self.item_table(rows.float())
        return pool_rows("final", table, off)


def get_final_attention_model(model_path: Optional[Path] = None) -> FinalAttention:
    """modeling_utils.py:274-279."""
    model = FinalAttention(reduced_dim=REDUCED_DIM, hidden_dim=FINAL_ATTENTION_HIDDEN_DIM)
    if model_path:
        model.load_state_dict(torch.load(model_path, weights_only=True))
    return model.to(DEVICE).eval()


def get_latent_attention_model(model_path: Optional[Path] = None) -> LatentAttentionModel:
    """modeling_utils.py:151-155."""
    model = LatentAttentionModel()
    if model_path:
        model.load_state_dict(torch.load(model_path, weights_only=True))
    return model.to(DEVICE).eval()


def normalize(x: torch.Tensor) -> torch.Tensor:
    return F.normalize(x, p=2, dim=1)
