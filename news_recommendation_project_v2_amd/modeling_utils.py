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

import numpy as np

import torch
import torch.nn.functional as F

from . import ops
from ._lib import NewsRecHIPError
from .attention import MyEncoder
from .config import DEVICE, EMBEDDING_DIM, FINAL_ATTENTION_HIDDEN_DIM, NUM_HIDDEN_LAYERS, REDUCED_DIM
from .latent_attention import LatentAttentionModel


def last_token_pool(last_hidden_states: torch.Tensor, attention_mask: torch.Tensor) -> torch.Tensor:
    """Hidden state of each row's last valid token (modeling_utils.py:37-48):
    if every row's last mask slot is set (left padding) take [:, -1], else
    index mask.sum - 1."""
    if bool((attention_mask[:, -1].sum() == attention_mask.shape[0]).item()):
        return last_hidden_states[:, -1]
    last = attention_mask.sum(dim=1) - 1
    return last_hidden_states[torch.arange(last_hidden_states.shape[0], device=last_hidden_states.device), last]


def last_token_rows(attention_mask: torch.Tensor) -> torch.Tensor:
    """Flat row index (b * L + position) that ``last_token_pool`` selects per row,
    with its exact semantics (modeling_utils.py:37-48): position L-1 for all rows
    when every row's last mask slot is set, else ``mask.sum - 1`` (an all-zero
    row gives -1, which torch indexing wraps to L-1)."""
    B, L = attention_mask.shape
    if bool((attention_mask[:, -1].sum() == B).item()):
        pos = torch.full((B,), L - 1, dtype=torch.int64, device=attention_mask.device)
    else:
        pos = (attention_mask.sum(dim=1).to(torch.int64) - 1) % L
    return torch.arange(B, device=attention_mask.device, dtype=torch.int64) * L + pos


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
    return ops.pool_rows(pooler, table, hist_off)


def _pad64(n: int) -> int:
    return max(64, (n + 63) // 64 * 64)


class _FinalAttentionFn(torch.autograd.Function):
    """FinalAttention forward + backward on the HIP kernels, over the packed valid
    history rows (CSR ``off``), so the reference module trains through autograd
    (trainer.py:1046-1063: ``model.train()``, forward, ``loss.backward()``).

    Forward (modeling_utils.py:218-228, f32, exact-f32 MFMA): rows padded with
    zeros to a multiple of 64 (the weight-grad GEMMs' K), then
      X1 = drop1(relu(S W1ᵀ + b1)); X2 = drop2(relu(X1 W2ᵀ + b2)); X = X2 W3ᵀ + b3
      Y = drop3(relu(X W4ᵀ + b4)); P = exp(Y W5ᵀ); users = Σ x p / (Σ p + 1e-10)
    with dropout fused into the ReLU epilogues (nr_gemm_relu_dropout: the
    counter-hash stream keyed by (seed, packed row, column), the same draw
    oracle/train_ref.py restates; p = 0 in eval).  Backward: nr_final_pool_bwd,
    data-grad GEMMs through transposed weights with the relu/dropout backward
    fused (nr_gemm_drelu), weight grads dOutᵀ · X as one grouped launch, bias
    grads by column sums; the padding rows carry zero gradient."""

    @staticmethod
    def forward(ctx, rows, off, ps, seeds, W1, b1, W2, b2, W3, b3, W4, b4, W5):
        Hs, D = rows.shape
        H = W1.shape[0]
        Hp = _pad64(Hs)
        dev = rows.device
        S = torch.zeros((Hp, D), dtype=torch.float32, device=dev)
        S[:Hs] = rows
        X1 = ops.gemm_relu_dropout(S, W1.contiguous(), b1.contiguous(), seeds[0], ps[0])
        X2 = ops.gemm_relu_dropout(X1, W2.contiguous(), b2.contiguous(), seeds[1], ps[1])
        XP = torch.empty((Hp, 2 * D), dtype=torch.float32, device=dev)
        X = XP[:, :D]
        ops.gemm(X2, W3.contiguous(), b3.contiguous(), out=X)
        Y = ops.gemm_relu_dropout(X, W4.contiguous(), b4.contiguous(), seeds[2], ps[2])
        ops.gemm(Y, W5.contiguous(), None, epilogue="exp", out=XP[:, D:])
        users, z = ops.final_pool_fwd(XP, off)
        ctx.save_for_backward(S, X1, X2, XP, Y, users, z, off, W1, W2, W3, W4, W5)
        ctx.ps, ctx.Hs = ps, Hs
        return users

    @staticmethod
    def backward(ctx, du):
        S, X1, X2, XP, Y, users, z, off, W1, W2, W3, W4, W5 = ctx.saved_tensors
        ps, Hs = ctx.ps, ctx.Hs
        Hp, D = S.shape
        du = du.float().contiguous()
        dXp = torch.empty((Hp, D), dtype=torch.float32, device=S.device)
        dL = torch.empty_like(dXp)
        ops.final_pool_bwd(XP, off, users, z, du, dXp, dL)
        X = XP[:, :D]
        T = ops.transpose
        dY = ops.gemm_drelu(dL, T(W5.contiguous()), Y, 1.0 / (1.0 - ps[2]))
        dX = ops.gemm(dY, T(W4.contiguous()), None, epilogue="resadd", residual=dXp)
        dZ2 = ops.gemm_drelu(dX, T(W3.contiguous()), X2, 1.0 / (1.0 - ps[1]))
        dZ1 = ops.gemm_drelu(dZ2, T(W2.contiguous()), X1, 1.0 / (1.0 - ps[0]))
        dS = ops.gemm(dZ1, T(W1.contiguous()), None)
        gW = [torch.empty_like(w, dtype=torch.float32) for w in (W1, W2, W3, W4, W5)]
        ops.gemm_grouped([(T(g_out), T(x_in), gw) for g_out, x_in, gw in
                          ((dZ1, S, gW[0]), (dZ2, X1, gW[1]), (dX, X2, gW[2]), (dY, X, gW[3]), (dL, Y, gW[4]))])
        gb = []
        for g_out in (dZ1, dZ2, dX, dY):
            b = torch.zeros(g_out.shape[1], dtype=torch.float32, device=S.device)
            ops.col_sum(g_out, b)
            gb.append(b)
        return (dS[:Hs], None, None, None, gW[0], gb[0], gW[1], gb[1], gW[2], gb[2], gW[3], gb[3], gW[4])


class FinalAttention(torch.nn.Module):
    """Additive per-dimension attention pooler (modeling_utils.py:175-228).

    forward(emb [B, L, D], mask [B, L]) -> [B, D]:
      x = W3 relu(W2 relu(W1 e + b1) + b2) + b3 ;  w = W5 relu(W4 x + b4)
      out = sum_L x * exp(w) * m / (sum_L exp(w) * m + 1e-10)
    In eval under no_grad: the per-item table once per valid row + the pooling
    kernel.  When autograd is recording (train mode, or any input / parameter
    requiring grad), ``_FinalAttentionFn``: the same math with the backward
    wired to the HIP kernels; in train mode the dropouts (p = 0.1, their
    modules' ``p``) are active, drawn from the counter-hash stream with seeds
    taken from torch's default generator (torch.manual_seed reproduces them).
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
        rows, off = flatten_valid(embeddings, attention_mask)
        params = [self.linear1.weight, self.linear1.bias, self.linear2.weight, self.linear2.bias, self.linear3.weight,
                  self.linear3.bias, self.linear4.weight, self.linear4.bias, self.linear5.weight]
        if self.training or (torch.is_grad_enabled() and (rows.requires_grad or any(p.requires_grad for p in params))):
            if any(p.dtype != torch.float32 for p in params):
                raise NewsRecHIPError("FinalAttention autograd path trains f32 parameters (as the reference does)")
            drops = (self.dropout1, self.dropout2, self.dropout3)
            ps = tuple(float(d.p) if self.training else 0.0 for d in drops)
            seeds = tuple(int(s) for s in torch.randint(0, 2**62, (3,)).tolist()) if self.training else (0, 0, 0)
            return _FinalAttentionFn.apply(rows.float(), off, ps, seeds, *params)
        table = self.item_table(rows.float())
        return pool_rows("final", table, off)


class FirstAttentionPoolFunc(torch.nn.Module):
    """Token-attention encoder + pooling (modeling_utils.py:498-513).

    ``self.encoder`` is the reference's ``MyEncoder`` (same state-dict keys),
    whose output is a chain of g_mlp_layernorms of its input (attention.py:193).
    With ``last_token_pool`` the whole forward is one gathered LayerNorm of each
    row's last valid token (``nr_gather_layernorm``): only B rows are read.
    Other pool functions get the full LN'd sequence.
    """

    def __init__(self, pool_func, embedding_dim=EMBEDDING_DIM, num_layers=NUM_HIDDEN_LAYERS):
        super().__init__()
        self.pool_func = pool_func
        self.encoder = MyEncoder(hidden_size=embedding_dim, num_hidden_layers=num_layers)

    def forward(self, embeddings: torch.Tensor, attention_mask: torch.Tensor) -> torch.Tensor:
        if embeddings.device.type != "cuda":
            raise NewsRecHIPError("FirstAttentionPoolFunc runs on the MI355X HIP path only (got a CPU tensor)")
        if self.pool_func is last_token_pool:
            rows = last_token_rows(attention_mask)
            return MyEncoder.ln_chain(list(self.encoder.layer), embeddings, row_idx=rows)
        return self.pool_func(self.encoder(embeddings, attention_mask), attention_mask)

    def forward_packed(self, rows: torch.Tensor, seg_off: torch.Tensor) -> torch.Tensor:
        """Packed variant: ``rows`` [T, D] holds every sequence's valid tokens back
        to back, ``seg_off`` [B+1] int64 the offsets; returns the last_token_pool
        output [B, D] f32 (each sequence must have >= 1 token)."""
        if self.pool_func is not last_token_pool:
            raise NewsRecHIPError("forward_packed implements last_token_pool only")
        last = (seg_off[1:] - 1).to(torch.int64).contiguous()
        return MyEncoder.ln_chain(list(self.encoder.layer), rows, row_idx=last)


def get_token_attn_model(model_path: Optional[Path] = None) -> FirstAttentionPoolFunc:
    """modeling_utils.py:516-524."""
    model = FirstAttentionPoolFunc(pool_func=last_token_pool, embedding_dim=EMBEDDING_DIM,
                                   num_layers=NUM_HIDDEN_LAYERS)
    if model_path:
        model.load_state_dict(torch.load(model_path, weights_only=True))
    return model.to(DEVICE)


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


# ---------------------------------------------------------------- title encoder API
# The reference's encoder entry points (modeling_utils.py:62-103, 282-323), kept
# by name and argument meaning over the packed-varlen HIP encoder (encoder.py):
# the HF model object becomes an ``XLMREncoder``; batches stay the tokenizer's
# right-padded ``input_ids`` / ``attention_mask``; pooling happens on the device.

def output_pool(model):
    """Pooling function of an encoder (modeling_utils.py:62-75): average_pool for
    the XLM-R architecture (e5-large-instruct), the only one on the HIP path;
    Qwen2 / NewModel / NV-Embed are out of scope and raise."""
    from .encoder import XLMREncoder
    if isinstance(model, XLMREncoder):
        return average_pool
    raise NotImplementedError(f"output_pool: {type(model).__name__} is not an XLM-R encoder on the HIP path")


def get_model_and_tokenizer(path: str, device=DEVICE, dtype: torch.dtype = torch.float32):
    """(encoder, tokenizer) for a LOCAL XLM-R directory (modeling_utils.py:92-103;
    no hub download).  ``dtype`` is the compute dtype of the HIP encoder (f32 for
    BASELINE config 2; bf16 for throughput)."""
    from transformers import AutoTokenizer

    from .encoder import XLMREncoder
    model = XLMREncoder.from_pretrained_dir(path, dtype=dtype, device=torch.device(device))
    return model, AutoTokenizer.from_pretrained(path)


def get_text_embed_eval(model, input_dataloader) -> torch.Tensor:
    """average_pool(last_hidden_state) of every batch, concatenated on the host
    (modeling_utils.py:282-300).  Each batch is a mapping with right-padded
    ``input_ids`` and ``attention_mask`` (eval_collate_fn's BatchEncoding); the
    padded slots are dropped and the sequences run packed through
    nr_encoder_forward, so only [B, 1024] leaves the device."""
    output_pool(model)  # architecture check, as the reference selects its pool here
    out = [model.encode_padded(inputs["input_ids"], inputs["attention_mask"]).cpu() for inputs in input_dataloader]
    return torch.cat(out) if out else torch.zeros((0, EMBEDDING_DIM))


def get_embed_from_model(model, text_dataset, text_maxlen: int, text_collate_fn,
                         batch_size: int = 1024) -> torch.Tensor:
    """modeling_utils.py:304-323: a sequential DataLoader over the texts, then
    get_text_embed_eval.  The reference sizes its batch by a GPU-OOM probe; here
    the batch only sets how many sequences the host tokenises at a time (the
    device works on packed tokens in chunks of ``model.max_tokens``)."""
    from torch.utils.data import DataLoader
    del text_maxlen  # applied by text_collate_fn (eval_collate_fn's max_len)
    loader = DataLoader(text_dataset, batch_size=batch_size, collate_fn=text_collate_fn, shuffle=False)
    return get_text_embed_eval(model, loader)


def get_model_eval(dataloader, model: torch.nn.Module) -> torch.Tensor:
    """Model outputs over a DataLoader, concatenated on the host (modeling_utils.py:402-417):
    tuple / list batches are unpacked as positional arguments."""
    out = []
    model.eval()
    with torch.no_grad():
        for item in dataloader:
            if isinstance(item, (tuple, list)):
                out.append(model(*(x.to(DEVICE) for x in item)).detach().cpu())
            else:
                out.append(model(item.to(DEVICE)).detach().cpu())
    return torch.cat(out)


def store_text_embed_full_eval(model, input_dataloader, db_name) -> int:
    """Per-token hidden states of every title into the sqlite token DB
    (modeling_utils.py:456-473): batches are the tokenizer's right-padded
    ``input_ids`` / ``attention_mask``; the valid tokens of each row are packed
    and run through the HIP encoder, and each row's [L_valid, 1024] states are
    stored fp16, ids 1.. in dataloader order (encoder.store_token_states)."""
    from .encoder import store_token_states
    ids, lens = [], []
    for inputs in input_dataloader:
        mask = torch.as_tensor(inputs["attention_mask"]).bool()
        ii = torch.as_tensor(inputs["input_ids"])
        ids.append(ii[mask].to(torch.int32).numpy())
        lens.append(mask.sum(1).to(torch.int64).numpy())
    flat = np.concatenate(ids) if ids else np.zeros(0, np.int32)
    return store_token_states(model, flat, np.concatenate(lens) if lens else np.zeros(0, np.int64), db_name)


def store_embed_from_model(model, text_dataset, text_maxlen: int, text_collate_fn, db_name,
                           batch_size: int = 1024) -> int:
    """modeling_utils.py:477-495: a sequential DataLoader over the texts, then
    store_text_embed_full_eval (the batch only sets host tokenisation chunks)."""
    from torch.utils.data import DataLoader
    del text_maxlen  # applied by text_collate_fn
    loader = DataLoader(text_dataset, batch_size=batch_size, collate_fn=text_collate_fn, shuffle=False)
    return store_text_embed_full_eval(model, loader, db_name)


# The classification-head / weighted-sum / reducing / NV-Embed experiments
# (modeling_utils.py:85-89, 106-172, 326-399, 420-453) are outside the hot path
# (DESIGN §7): import-level placeholders only.
from .out_of_scope import placeholder_class as _oos_cls, placeholder_function as _oos_fn  # noqa: E402

get_nvembed_model = _oos_fn("get_nvembed_model", "modeling_utils.py:85-89", __name__)
get_nv_embeds = _oos_fn("get_nv_embeds", "modeling_utils.py:371-399", __name__)
ClassificationHead = _oos_cls("ClassificationHead", "modeling_utils.py:106-116", __name__, torch.nn.Module)
ClassificationHeadCatEmbed = _oos_cls("ClassificationHeadCatEmbed", "modeling_utils.py:119-136", __name__,
                                      torch.nn.Module)
get_classification_head = _oos_fn("get_classification_head", "modeling_utils.py:139-148", __name__)
WeightedSumModel = _oos_cls("WeightedSumModel", "modeling_utils.py:158-165", __name__, torch.nn.Module)
get_weighted_sum_model = _oos_fn("get_weighted_sum_model", "modeling_utils.py:168-172", __name__)
EmbeddingWrapper = _oos_cls("EmbeddingWrapper", "modeling_utils.py:326-340", __name__, torch.nn.Module)
get_embed_wrapped_model = _oos_fn("get_embed_wrapped_model", "modeling_utils.py:343-346", __name__)
ResizeWrapperModel = _oos_cls("ResizeWrapperModel", "modeling_utils.py:349-364", __name__, torch.nn.Module)
resize_wrap_model = _oos_fn("resize_wrap_model", "modeling_utils.py:367-368", __name__)
get_head_model = _oos_fn("get_head_model", "modeling_utils.py:420-427", __name__)
get_new_attention_model = _oos_fn("get_new_attention_model", "modeling_utils.py:430-435", __name__)
ReducingModel = _oos_cls("ReducingModel", "modeling_utils.py:438-446", __name__, torch.nn.Module)
get_reducing_model = _oos_fn("get_reducing_model", "modeling_utils.py:449-453", __name__)
