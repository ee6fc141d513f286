"""Tensor-level wrappers over the C-ABI (include/newsrec.h).

Every function takes device tensors (PyTorch-ROCm "cuda" tensors), validates
shapes/dtypes/strides on the host, and enqueues the HIP kernel on the current
torch stream.  There is no CPU fallback: non-device tensors raise.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch

from . import _lib

_DT = {torch.float32: _lib.NR_F32, torch.bfloat16: _lib.NR_BF16}
_EPI = {
    "none": _lib.NR_EPI_NONE,
    "relu": _lib.NR_EPI_RELU,
    "exp": _lib.NR_EPI_EXP,
    "geglu": _lib.NR_EPI_GEGLU,
    "resadd": _lib.NR_EPI_RESADD,
    "gelu": _lib.NR_EPI_GELU,
    "softmax64": _lib.NR_EPI_SOFTMAX64,
    "softmax64_bwd": _lib.NR_EPI_SOFTMAX64_BWD,  # residual = the softmax output P
}
POOLERS = {"final": _lib.NR_POOL_FINAL, "latent": _lib.NR_POOL_LATENT, "mean": _lib.NR_POOL_MEAN}


def _ptr(t: Optional[torch.Tensor]):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _stream(dev: torch.device):
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def _dev(*ts: Optional[torch.Tensor]) -> torch.device:
    dev = None
    for t in ts:
        if t is None:
            continue
        if t.device.type != "cuda":
            raise _lib.NewsRecHIPError(
                f"HIP kernels need device tensors, got a tensor on {t.device} (no CPU fallback)")
        if dev is None:
            dev = t.device
        elif t.device != dev:
            raise _lib.NewsRecHIPError(f"tensors on different devices: {dev} vs {t.device}")
    return dev


def _rowmajor(t: torch.Tensor, name: str) -> int:
    if t.dim() != 2 or t.stride(1) != 1:
        raise _lib.NewsRecHIPError(f"{name} must be a row-major 2-D tensor (stride(1)==1)")
    return t.stride(0)


def _dtype(t: torch.Tensor, name: str) -> int:
    if t.dtype not in _DT:
        raise _lib.NewsRecHIPError(f"{name}: unsupported dtype {t.dtype}")
    return _DT[t.dtype]


def set_persistent_workgroups(n: int = 0) -> None:
    """Workgroups of the persistent bf16 GEMM launches (0 = one per CU): set it
    to the CU count of a CU-masked stream the transform runs on."""
    _lib.call("nr_set_persistent_workgroups", int(n))


def persistent_workgroups() -> int:
    """The current persistent-GEMM workgroup budget (0 = one per CU)."""
    return int(_lib.load().nr_persistent_workgroups())


def set_gemm_half_tail(on: bool = True) -> None:
    """Half-tile tail of the persistent bf16 GEMM (default on; bit-identical
    either way -- the switch is for A/B timing)."""
    _lib.call("nr_set_gemm_half_tail", int(bool(on)))


def gemm(a: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None,
         epilogue: str = "none", residual: Optional[torch.Tensor] = None,
         out: Optional[torch.Tensor] = None, out_dtype: Optional[torch.dtype] = None) -> torch.Tensor:
    """out = epilogue(a @ w.T + bias [+ residual]); w in nn.Linear layout [N, K]."""
    dev = _dev(a, w, bias, residual, out)
    if a.dtype != w.dtype:
        raise _lib.NewsRecHIPError("gemm: a and w must share a dtype")
    M, K = a.shape
    N, K2 = w.shape
    if K != K2:
        raise _lib.NewsRecHIPError(f"gemm: K mismatch {K} vs {K2}")
    epi = _EPI[epilogue]
    ncols = N // 2 if epilogue == "geglu" else N
    if out is None:
        out = torch.empty((M, ncols), dtype=out_dtype or a.dtype, device=dev)
    if bias is not None and (bias.dtype != torch.float32 or not bias.is_contiguous() or bias.numel() != N):
        raise _lib.NewsRecHIPError("gemm: bias must be contiguous f32 [N]")
    if residual is not None and residual.dtype != out.dtype:
        raise _lib.NewsRecHIPError("gemm: residual must have the output dtype")
    if out.shape != (M, ncols):
        raise _lib.NewsRecHIPError(f"gemm: out shape {tuple(out.shape)} != {(M, ncols)}")
    lda, ldw, ldc = _rowmajor(a, "a"), _rowmajor(w, "w"), _rowmajor(out, "out")
    ldr = _rowmajor(residual, "residual") if residual is not None else 0
    _lib.call("nr_gemm", _dtype(a, "a"), _dtype(out, "out"), epi, M, N, K, _ptr(a), lda, _ptr(w), ldw,
              _ptr(bias), _ptr(residual), ldr, _ptr(out), ldc, _stream(dev))
    return out


def layernorm(x: torch.Tensor, gamma: Optional[torch.Tensor], beta: Optional[torch.Tensor], eps: float,
              out: Optional[torch.Tensor] = None, out_dtype: Optional[torch.dtype] = None) -> torch.Tensor:
    dev = _dev(x, gamma, beta, out)
    rows, dim = x.shape
    if out is None:
        out = torch.empty((rows, dim), dtype=out_dtype or x.dtype, device=dev)
    _lib.call("nr_layernorm", _dtype(x, "x"), _dtype(out, "out"), rows, dim, _ptr(x), _rowmajor(x, "x"),
              _ptr(gamma), _ptr(beta), ctypes.c_float(eps), _ptr(out), _rowmajor(out, "out"), _stream(dev))
    return out


def gather_layernorm(x: torch.Tensor, row_idx: Optional[torch.Tensor], gammas: Optional[torch.Tensor],
                     betas: Optional[torch.Tensor], eps: float, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out[i] = LN chain (gammas/betas [n_ln, D]) of x[row_idx[i]] (identity if None), f32 out.

    x may be f32, bf16 or f16 (the token-state blobs are fp16)."""
    dev = _dev(x, row_idx, gammas, betas, out)
    if x.dim() != 2 or x.stride(1) != 1:
        raise _lib.NewsRecHIPError("gather_layernorm: x must be row-major 2-D")
    dt = {torch.float32: _lib.NR_F32, torch.bfloat16: _lib.NR_BF16, torch.float16: _lib.NR_F16}.get(x.dtype)
    if dt is None:
        raise _lib.NewsRecHIPError(f"gather_layernorm: unsupported dtype {x.dtype}")
    dim = x.shape[1]
    if row_idx is not None:
        if row_idx.dtype != torch.int64 or not row_idx.is_contiguous():
            raise _lib.NewsRecHIPError("gather_layernorm: row_idx must be contiguous int64")
        n = row_idx.numel()
    else:
        n = x.shape[0]
    n_ln = 0
    for t in (gammas, betas):
        if t is not None:
            if t.dtype != torch.float32 or not t.is_contiguous() or t.dim() != 2 or t.shape[1] != dim:
                raise _lib.NewsRecHIPError("gather_layernorm: gammas/betas must be contiguous f32 [n_ln, D]")
            n_ln = max(n_ln, t.shape[0])
    if gammas is not None and betas is not None and gammas.shape != betas.shape:
        raise _lib.NewsRecHIPError("gather_layernorm: gammas and betas differ in shape")
    if out is None:
        out = torch.empty((n, dim), dtype=torch.float32, device=dev)
    if out.dtype != torch.float32 or out.shape != (n, dim):
        raise _lib.NewsRecHIPError("gather_layernorm: out must be f32 [n, D]")
    _lib.call("nr_gather_layernorm", dt, n, dim, _ptr(x), x.stride(0), _ptr(row_idx), n_ln, _ptr(gammas),
              _ptr(betas), ctypes.c_float(eps), _ptr(out), _rowmajor(out, "out"), _stream(dev))
    return out


def softmax64(x: torch.Tensor, out: Optional[torch.Tensor] = None,
              out_dtype: Optional[torch.dtype] = None) -> torch.Tensor:
    dev = _dev(x, out)
    if x.dtype != torch.float32:
        raise _lib.NewsRecHIPError("softmax64: x must be f32")
    rows, width = x.shape
    if width % 64:
        raise _lib.NewsRecHIPError("softmax64: width must be a multiple of 64")
    if out is None:
        out = torch.empty((rows, width), dtype=out_dtype or torch.float32, device=dev)
    _lib.call("nr_softmax64", rows, width // 64, _ptr(x), _rowmajor(x, "x"), _dtype(out, "out"), _ptr(out),
              _rowmajor(out, "out"), _stream(dev))
    return out


def row_inv_norm(x: torch.Tensor, eps: float = 1e-8, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """1 / max(||x_r||, eps) per row, f32 (cosine_similarity's per-vector clamp)."""
    dev = _dev(x, out)
    rows, dim = x.shape
    if out is None:
        out = torch.empty(rows, dtype=torch.float32, device=dev)
    _lib.call("nr_row_inv_norm", _dtype(x, "x"), rows, dim, _ptr(x), _rowmajor(x, "x"), ctypes.c_float(eps),
              _ptr(out), _stream(dev))
    return out


def row_stats(x: torch.Tensor, eps: float = 1e-5, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Per-row LayerNorm statistics [rows, 2] f32 = (mean, 1/sqrt(biased var + eps))."""
    dev = _dev(x, out)
    rows, dim = x.shape
    if out is None:
        out = torch.empty((rows, 2), dtype=torch.float32, device=dev)
    _lib.call("nr_row_stats", _dtype(x, "x"), rows, dim, _ptr(x), _rowmajor(x, "x"), ctypes.c_float(eps),
              _ptr(out), _stream(dev))
    return out


def _check_csr(idx: torch.Tensor, off: torch.Tensor, name: str) -> None:
    if idx.dtype != torch.int32 or not idx.is_contiguous():
        raise _lib.NewsRecHIPError(f"{name}_idx must be contiguous int32")
    if off.dtype != torch.int64 or not off.is_contiguous():
        raise _lib.NewsRecHIPError(f"{name}_off must be contiguous int64")


def pool_score(pooler: str, hist_table: torch.Tensor, cand_table: torch.Tensor, cand_inv_norm: torch.Tensor,
               hist_idx: torch.Tensor, hist_off: torch.Tensor, cand_idx: torch.Tensor, cand_off: torch.Tensor,
               n_cand: int, want_users: bool = False, scores: Optional[torch.Tensor] = None):
    """Fused history pooling + cosine scoring; returns (scores[C] f32, users[I, D] f32 or None).

    ``n_cand`` = cand_off[-1] (passed by the caller so no device sync is needed).
    """
    dev = _dev(hist_table, cand_table, cand_inv_norm, hist_idx, hist_off, cand_idx, cand_off, scores)
    _check_csr(hist_idx, hist_off, "hist")
    _check_csr(cand_idx, cand_off, "cand")
    if hist_off.numel() != cand_off.numel():
        raise _lib.NewsRecHIPError("hist_off and cand_off must both have n_imp + 1 entries")
    if hist_table.dtype != cand_table.dtype:
        raise _lib.NewsRecHIPError("hist_table and cand_table must share a dtype")
    if cand_inv_norm.dtype != torch.float32 or cand_inv_norm.numel() < cand_table.shape[0]:
        raise _lib.NewsRecHIPError("cand_inv_norm must be f32 with one entry per candidate-table row")
    n_imp = hist_off.numel() - 1
    dim = cand_table.shape[1]
    # empty CSR arrays have no storage; the kernel never reads them (offsets are
    # all equal) but the C-ABI rejects null pointers, so hand it a 1-slot dummy
    one = None
    if hist_idx.numel() == 0 or cand_idx.numel() == 0 or n_cand == 0:
        one = torch.zeros(1, dtype=torch.int32, device=dev)
    if hist_idx.numel() == 0:
        hist_idx = one
    if cand_idx.numel() == 0:
        cand_idx = one
    if scores is None:
        scores = torch.empty(n_cand, dtype=torch.float32, device=dev)
    # zero-element tensors report data_ptr() == 0: give the kernel a real (unread) slot
    scores_buf = scores if scores.numel() > 0 else torch.empty(1, dtype=torch.float32, device=dev)
    users = torch.empty((n_imp, dim), dtype=torch.float32, device=dev) if want_users else None
    _lib.call("nr_pool_score", POOLERS[pooler], _dtype(cand_table, "cand_table"), dim, _ptr(hist_table),
              _rowmajor(hist_table, "hist_table"), _ptr(cand_table), _rowmajor(cand_table, "cand_table"),
              _ptr(cand_inv_norm), _ptr(hist_idx), _ptr(hist_off), _ptr(cand_idx), _ptr(cand_off), n_imp,
              _ptr(scores_buf), _ptr(users) if users is not None and users.numel() else None, _stream(dev))
    return scores, users


def pool_users(pooler: str, hist_table: torch.Tensor, hist_idx: torch.Tensor, hist_off: torch.Tensor,
               out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Pooling only (nr_pool_score with no candidates): users [n, D] f32, one
    row per history segment (into ``out`` when given)."""
    dev = _dev(hist_table, hist_idx, hist_off, out)
    _check_csr(hist_idx, hist_off, "hist")
    n, dim = hist_off.numel() - 1, hist_table.shape[1] if pooler != "final" else hist_table.shape[1] // 2
    if out is not None and (out.dtype != torch.float32 or out.shape != (n, dim) or not out.is_contiguous()):
        raise _lib.NewsRecHIPError(f"pool_users: out must be contiguous f32 {(n, dim)}")
    users = torch.empty((n, dim), dtype=torch.float32, device=dev) if out is None else out
    if n == 0:
        return users
    hidx = hist_idx if hist_idx.numel() else torch.zeros(1, dtype=torch.int32, device=dev)
    _lib.call("nr_pool_score", POOLERS[pooler], _dtype(hist_table, "hist_table"), dim, _ptr(hist_table),
              _rowmajor(hist_table, "hist_table"), None, 0, None, _ptr(hidx), _ptr(hist_off), None, None, n, None,
              _ptr(users), _stream(dev))
    return users


def score_users(users: torch.Tensor, user_idx: torch.Tensor, cand_table: torch.Tensor, cand_inv_norm: torch.Tensor,
                cand_idx: torch.Tensor, cand_off: torch.Tensor, n_cand: int,
                scores: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Scores of every impression's candidates against users[user_idx[i]]
    (nr_score_users); bit-identical to the fused pool_score pass."""
    dev = _dev(users, user_idx, cand_table, cand_inv_norm, cand_idx, cand_off, scores)
    _check_csr(cand_idx, cand_off, "cand")
    if users.dtype != torch.float32 or not users.is_contiguous() or user_idx.dtype != torch.int32:
        raise _lib.NewsRecHIPError("score_users: users contiguous f32, user_idx int32")
    if user_idx.numel() != cand_off.numel() - 1:
        raise _lib.NewsRecHIPError("score_users: one user index per impression")
    if scores is None:
        scores = torch.empty(n_cand, dtype=torch.float32, device=dev)
    if n_cand == 0 or user_idx.numel() == 0:
        return scores
    _lib.call("nr_score_users", _dtype(cand_table, "cand_table"), cand_table.shape[1], _ptr(users), _ptr(user_idx),
              _ptr(cand_table), _rowmajor(cand_table, "cand_table"), _ptr(cand_inv_norm), _ptr(cand_idx),
              _ptr(cand_off), user_idx.numel(), _ptr(scores), _stream(dev))
    return scores


def dense_rank(scores: torch.Tensor, cand_off: torch.Tensor, check: bool = True) -> torch.Tensor:
    """Per-impression dense descending ranks (int32), scipy rankdata(-x, 'dense')."""
    dev = _dev(scores, cand_off)
    if scores.dtype != torch.float32 or not scores.is_contiguous():
        raise _lib.NewsRecHIPError("dense_rank: scores must be contiguous f32")
    ranks = torch.empty(scores.numel(), dtype=torch.int32, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    _lib.call("nr_dense_rank", _ptr(scores), _ptr(cand_off), cand_off.numel() - 1, _ptr(ranks), _ptr(status),
              _stream(dev))
    if check and int(status.item()) != 0:
        raise _lib.NewsRecHIPError("dense_rank: an impression has more than 2048 candidates")
    return ranks


def impression_metrics(ranks: torch.Tensor, labels: torch.Tensor, cand_off: torch.Tensor):
    """Per-impression (AUC, MRR, nDCG@5, nDCG@10) f64 [n, 4] + tie flags int32 [n]
    from dense ranks (int32) and 0/1 labels (f32); raises on >2048 candidates or
    non-binary labels."""
    dev = _dev(ranks, labels, cand_off)
    if ranks.dtype != torch.int32 or labels.dtype != torch.float32 or cand_off.dtype != torch.int64:
        raise _lib.NewsRecHIPError("impression_metrics: ranks int32, labels f32, cand_off int64")
    n = cand_off.numel() - 1
    out = torch.empty((n, 4), dtype=torch.float64, device=dev)
    tie = torch.empty(n, dtype=torch.int32, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    _lib.call("nr_impression_metrics", _ptr(ranks), _ptr(labels), _ptr(cand_off), n, _ptr(out), _ptr(tie),
              _ptr(status), _stream(dev))
    st = int(status.item())
    if st & 1:
        raise _lib.NewsRecHIPError("impression_metrics: an impression has more than 2048 candidates")
    if st & 2:
        raise _lib.NewsRecHIPError("impression_metrics: labels must be 0/1 and ranks in 1..c")
    return out, tie


def final_attn_transform(emb: torch.Tensor, w: dict, out: Optional[torch.Tensor] = None,
                         workspace: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Per-news FinalAttention table [n, 2*1024] = (x, exp(w)) in emb.dtype.

    ``w`` holds device weights in emb.dtype (W1..W5) and f32 biases (b1..b4).
    """
    dev = _dev(emb, out)
    dt = _dtype(emb, "emb")
    n, dim = emb.shape
    if dim != 1024:
        raise _lib.NewsRecHIPError("final_attn_transform: dim must be 1024")
    if out is None:
        out = torch.empty((n, 2 * dim), dtype=emb.dtype, device=dev)
    need = _lib.load().nr_final_attn_workspace_bytes(dt, n)
    if workspace is None or workspace.numel() * workspace.element_size() < need:
        workspace = torch.empty(need, dtype=torch.uint8, device=dev)
    for k in ("W1", "W2", "W3", "W4", "W5"):
        if w[k].dtype != emb.dtype or not w[k].is_contiguous():
            raise _lib.NewsRecHIPError(f"final_attn_transform: {k} must be contiguous {emb.dtype}")
    _lib.call("nr_final_attn_transform", dt, n, _ptr(emb), _rowmajor(emb, "emb"), _ptr(w["W1"]), _ptr(w["b1"]),
              _ptr(w["W2"]), _ptr(w["b2"]), _ptr(w["W3"]), _ptr(w["b3"]), _ptr(w["W4"]), _ptr(w["b4"]),
              _ptr(w["W5"]), _ptr(out), _ptr(workspace), need, _stream(dev))
    return out


def latent_transform(emb: torch.Tensor, w: dict, out: Optional[torch.Tensor] = None,
                     workspace: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Per-news LatentAttention table [n, 1024] (the pre-pooling hiddens)."""
    dev = _dev(emb, out)
    dt = _dtype(emb, "emb")
    n, dim = emb.shape
    if dim != 1024:
        raise _lib.NewsRecHIPError("latent_transform: dim must be 1024")
    if out is None:
        out = torch.empty((n, dim), dtype=emb.dtype, device=dev)
    need = _lib.load().nr_latent_workspace_bytes(dt, n)
    if workspace is None or workspace.numel() * workspace.element_size() < need:
        workspace = torch.empty(need, dtype=torch.uint8, device=dev)
    for k in ("A", "Bt", "W1i", "W2"):
        if w[k].dtype != emb.dtype or not w[k].is_contiguous():
            raise _lib.NewsRecHIPError(f"latent_transform: {k} must be contiguous {emb.dtype}")
    if dt == _lib.NR_BF16 and "Wq_ln" in w:
        # both LayerNorms folded into the GEMMs that consume them (latent_attention.lnfold_weights)
        _lib.call("nr_latent_transform_lnfold", dt, n, _ptr(emb), _rowmajor(emb, "emb"), _ptr(w["Wq_ln"]),
                  _ptr(w["ucq"]), _ptr(w["Bt"]), _ptr(w["Wf_ln"]), _ptr(w["ucf"]), _ptr(w["W2"]), _ptr(w["b2"]),
                  _ptr(out), _ptr(workspace), need, _stream(dev))
        return out
    _lib.call("nr_latent_transform", dt, n, _ptr(emb), _rowmajor(emb, "emb"), _ptr(w["lnq_g"]), _ptr(w["lnq_b"]),
              _ptr(w["A"]), _ptr(w["Bt"]), _ptr(w["lnf_g"]), _ptr(w["lnf_b"]), _ptr(w["W1i"]), _ptr(w["b1i"]),
              _ptr(w["W2"]), _ptr(w["b2"]), _ptr(out), _ptr(workspace), need, _stream(dev))
    return out


def embed_ln(ids: torch.Tensor, pos: torch.Tensor, word: torch.Tensor, pos_emb: torch.Tensor, type_emb: torch.Tensor,
             gamma: torch.Tensor, beta: torch.Tensor, eps: float, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """LN(word[ids] + type_emb + pos_emb[pos]) for packed token rows (XLM-R embeddings)."""
    dev = _dev(ids, pos, word, pos_emb, type_emb, gamma, beta, out)
    if ids.dtype != torch.int32 or pos.dtype != torch.int32:
        raise _lib.NewsRecHIPError("embed_ln: ids/pos must be int32")
    if word.shape[1] != 1024:
        raise _lib.NewsRecHIPError("embed_ln: hidden size must be 1024")
    n = ids.numel()
    if out is None:
        out = torch.empty((n, 1024), dtype=word.dtype, device=dev)
    _lib.call("nr_embed_ln", _dtype(word, "word"), n, _ptr(ids), _ptr(pos), _ptr(word), _ptr(pos_emb),
              _ptr(type_emb), _ptr(gamma), _ptr(beta), ctypes.c_float(eps), _ptr(out), _stream(dev))
    return out


def attention_varlen(qkv: torch.Tensor, cu_seqlens: torch.Tensor, qblock_off: torch.Tensor, n_qblocks: int,
                     out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """16-head x 64 self-attention per packed sequence: qkv [T, 3072] -> ctx [T, 1024]."""
    dev = _dev(qkv, cu_seqlens, qblock_off, out)
    if qkv.shape[1] != 3072 or not qkv.is_contiguous():
        raise _lib.NewsRecHIPError("attention_varlen: qkv must be contiguous [T, 3072]")
    if cu_seqlens.dtype != torch.int32 or qblock_off.dtype != torch.int32:
        raise _lib.NewsRecHIPError("attention_varlen: offsets must be int32")
    if out is None:
        out = torch.empty((qkv.shape[0], 1024), dtype=qkv.dtype, device=dev)
    _lib.call("nr_attention_varlen", _dtype(qkv, "qkv"), cu_seqlens.numel() - 1, n_qblocks, _ptr(qkv),
              _ptr(cu_seqlens), _ptr(qblock_off), _ptr(out), _stream(dev))
    return out


def pool_rows(pooler: str, table: torch.Tensor, off: torch.Tensor) -> torch.Tensor:
    """Pool consecutive rows per segment (segment i = rows off[i]..off[i+1]-1):
    users [n_seg, 1024] f32 ("mean" = average_pool, "latent" = + F.normalize,
    "final" = FinalAttention pooling of [x | exp(w)] rows)."""
    dev = _dev(table, off)
    if off.dtype != torch.int64 or not off.is_contiguous():
        raise _lib.NewsRecHIPError("pool_rows: off must be contiguous int64")
    n_seg = off.numel() - 1
    users = torch.empty((n_seg, 1024), dtype=torch.float32, device=dev)
    if n_seg == 0:
        return users
    _lib.call("nr_pool_score", POOLERS[pooler], _dtype(table, "table"), 1024, _ptr(table), _rowmajor(table, "table"),
              None, 0, None, None, _ptr(off), None, None, n_seg, None, _ptr(users), _stream(dev))
    return users


_ENC_POOL = {"mean": _lib.NR_POOL_MEAN, "normalize": _lib.NR_POOL_LATENT, None: _lib.NR_POOL_NONE}


def encoder_forward(layers, emb: dict, ids: torch.Tensor, seq_lens: torch.Tensor, n_tokens: int,
                    pool: Optional[str] = "mean", want_hidden: bool = False, eps: float = 1e-5,
                    workspace: Optional[torch.Tensor] = None, status: Optional[torch.Tensor] = None):
    """Whole XLM-R forward through ``nr_encoder_forward`` (one C-ABI call).

    layers: a ctypes array of ``_lib.EncoderLayer``; emb: word / pos / type
    embedding tensors (dtype of the weights) and LN gamma / beta (f32); ids
    int32 [n_tokens] and seq_lens int32 [n_seq] on the device.  Returns
    (pooled [n_seq, 1024] f32 or None, hidden [n_tokens, 1024] or None)."""
    dev = _dev(ids, seq_lens, emb["word"], workspace, status)
    if ids.dtype != torch.int32 or seq_lens.dtype != torch.int32 or not ids.is_contiguous():
        raise _lib.NewsRecHIPError("encoder_forward: ids / seq_lens must be contiguous int32")
    dt = _dtype(emb["word"], "word")
    n_seq = seq_lens.numel()
    pooled = torch.empty((n_seq, 1024), dtype=torch.float32, device=dev) if pool else None
    hidden = torch.empty((n_tokens, 1024), dtype=emb["word"].dtype, device=dev) if want_hidden else None
    need = _lib.load().nr_encoder_workspace_bytes(dt, n_tokens, n_seq)
    if workspace is None or workspace.numel() * workspace.element_size() < need:
        workspace = torch.empty(need, dtype=torch.uint8, device=dev)
    _lib.call("nr_encoder_forward", dt, len(layers), ctypes.cast(layers, ctypes.c_void_p) if len(layers) else None,
              _ptr(emb["word"]), emb["word"].shape[0], _ptr(emb["pos"]), emb["pos"].shape[0], _ptr(emb["type"]),
              _ptr(emb["ln_g"]), _ptr(emb["ln_b"]), ctypes.c_float(eps), n_seq, n_tokens, _ptr(seq_lens), _ptr(ids),
              _ENC_POOL[pool], _ptr(pooled), _ptr(hidden), _ptr(status), _ptr(workspace), need, _stream(dev))
    return pooled, hidden


# ------------------------------------------------------------------ training step (config 5)
def _dt(t: torch.Tensor, name: str) -> int:
    return _dtype(t, name)


def gemm_grouped(problems) -> None:
    """out_i = a_i @ w_i.T for up to 8 (a, w, out) triples in ONE launch over all
    their 256x256 tiles (nr_gemm_grouped): small GEMMs that cannot fill the
    chip alone run side by side.  bf16 or f32 a/w, f32 or bf16 out (one out dtype)."""
    problems = list(problems)
    if not 1 <= len(problems) <= 8:
        raise _lib.NewsRecHIPError("gemm_grouped: 1..8 problems")
    dev = _dev(*[t for pr in problems for t in pr])
    n = len(problems)
    L = ctypes.c_int64 * n
    P = ctypes.c_void_p * n
    M, N, K, lda, ldw, ldc = L(), L(), L(), L(), L(), L()
    A, W, C = P(), P(), P()
    for i, (a, w, out) in enumerate(problems):
        if a.dtype != w.dtype or a.shape[1] != w.shape[1] or tuple(out.shape) != (a.shape[0], w.shape[0]):
            raise _lib.NewsRecHIPError(f"gemm_grouped: problem {i} shape/dtype mismatch")
        if out.dtype != problems[0][2].dtype:
            raise _lib.NewsRecHIPError("gemm_grouped: all outputs must share a dtype")
        M[i], K[i], N[i] = a.shape[0], a.shape[1], w.shape[0]
        lda[i], ldw[i], ldc[i] = _rowmajor(a, "a"), _rowmajor(w, "w"), _rowmajor(out, "out")
        A[i], W[i], C[i] = a.data_ptr(), w.data_ptr(), out.data_ptr()
    _lib.call("nr_gemm_grouped", _dtype(problems[0][0], "a"), _dtype(problems[0][2], "out"), n, M, N, K, A, lda, W,
              ldw, C, ldc, _stream(dev))


def gemm_grouped_tn(problems, alpha=None) -> None:
    """out_i = alpha_i * a_i.T @ w_i for up to 8 (a, w, out) triples in ONE launch
    (nr_gemm_grouped_tn): a_i [K, M], w_i [K, N] bf16 row-major (the weight grads
    dOut^T X straight from the activations), out_i [M, N] f32 or bf16."""
    problems = list(problems)
    if not 1 <= len(problems) <= 8:
        raise _lib.NewsRecHIPError("gemm_grouped_tn: 1..8 problems")
    dev = _dev(*[t for pr in problems for t in pr])
    n = len(problems)
    L = ctypes.c_int64 * n
    P = ctypes.c_void_p * n
    M, N, K, lda, ldw, ldc = L(), L(), L(), L(), L(), L()
    A, W, C = P(), P(), P()
    al = (ctypes.c_float * n)(*([1.0] * n if alpha is None else alpha))
    for i, (a, w, out) in enumerate(problems):
        if a.dtype != torch.bfloat16 or w.dtype != torch.bfloat16 or a.shape[0] != w.shape[0] \
                or tuple(out.shape) != (a.shape[1], w.shape[1]):
            raise _lib.NewsRecHIPError(f"gemm_grouped_tn: problem {i} shape/dtype mismatch")
        if out.dtype != problems[0][2].dtype:
            raise _lib.NewsRecHIPError("gemm_grouped_tn: all outputs must share a dtype")
        K[i], M[i], N[i] = a.shape[0], a.shape[1], w.shape[1]
        lda[i], ldw[i], ldc[i] = _rowmajor(a, "a"), _rowmajor(w, "w"), _rowmajor(out, "out")
        A[i], W[i], C[i] = a.data_ptr(), w.data_ptr(), out.data_ptr()
    _lib.call("nr_gemm_grouped_tn", _dtype(problems[0][2], "out"), n, M, N, K, A, lda, W, ldw, C, ldc, al,
              _stream(dev))


def gemm_relu_dropout(a: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor], seed: int, p: float,
                      out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out = relu(a @ w.T + bias) * keep / (1 - p), keep from the (seed, row, col) hash stream."""
    dev = _dev(a, w, bias, out)
    M, K = a.shape
    N = w.shape[0]
    if out is None:
        out = torch.empty((M, N), dtype=a.dtype, device=dev)
    _lib.call("nr_gemm_relu_dropout", _dt(a, "a"), _dt(out, "out"), M, N, K, _ptr(a), _rowmajor(a, "a"), _ptr(w),
              _rowmajor(w, "w"), _ptr(bias), _ptr(out), _rowmajor(out, "out"), ctypes.c_uint64(seed & (2**64 - 1)),
              ctypes.c_float(p), _stream(dev))
    return out


def gemm_drelu(a: torch.Tensor, w: torch.Tensor, y: torch.Tensor, scale: float,
               out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out = (y > 0) ? (a @ w.T) * scale : 0 (backward of relu + dropout, y = forward output)."""
    dev = _dev(a, w, y, out)
    M, K = a.shape
    N = w.shape[0]
    if out is None:
        out = torch.empty((M, N), dtype=y.dtype, device=dev)
    _lib.call("nr_gemm_drelu", _dt(a, "a"), _dt(out, "out"), M, N, K, _ptr(a), _rowmajor(a, "a"), _ptr(w),
              _rowmajor(w, "w"), _ptr(y), _rowmajor(y, "y"), _ptr(out), _rowmajor(out, "out"), ctypes.c_float(scale),
              _stream(dev))
    return out


def splitk_fixup(partials: torch.Tensor, out: torch.Tensor, epilogue: str = "none", bias: Optional[torch.Tensor] = None,
                 residual: Optional[torch.Tensor] = None, row0: int = 0, seed: int = 0, p: float = 0.0,
                 scale: float = 1.0) -> torch.Tensor:
    """out = epi(partials.sum(0) + bias) for K-slice partials [parts, rows, N] f32
    (nr_splitk_fixup): epilogue "none", "relu_dropout" (mask rows row0..), "drelu"
    (residual = the forward output), "resadd" (+ residual) or "exp"."""
    dev = _dev(partials, out, bias, residual)
    epi = {"none": _lib.NR_EPI_NONE, "relu_dropout": _lib.NR_EPI_RELU_DROPOUT, "drelu": _lib.NR_EPI_DRELU,
           "resadd": _lib.NR_EPI_RESADD, "exp": _lib.NR_EPI_EXP}[epilogue]
    if partials.dtype != torch.float32 or not partials.is_contiguous() or partials.dim() != 3:
        raise _lib.NewsRecHIPError("splitk_fixup: partials must be contiguous f32 [parts, rows, N]")
    parts, rows, N = partials.shape
    if tuple(out.shape) != (rows, N):
        raise _lib.NewsRecHIPError("splitk_fixup: out must be [rows, N]")
    _lib.call("nr_splitk_fixup", _dt(out, "out"), epi, rows, N, parts, _ptr(partials), _ptr(bias), _ptr(residual),
              _rowmajor(residual, "residual") if residual is not None else 0, _ptr(out), _rowmajor(out, "out"), row0,
              ctypes.c_uint64(seed & (2**64 - 1)), ctypes.c_float(p), ctypes.c_float(scale), _stream(dev))
    return out


def gather_rows(src: torch.Tensor, idx: Optional[torch.Tensor], n: Optional[int] = None,
                out_dtype: Optional[torch.dtype] = None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    dev = _dev(src, idx, out)
    n = idx.numel() if idx is not None else (n if n is not None else src.shape[0])
    if idx is not None and (idx.dtype != torch.int32 or not idx.is_contiguous()):
        raise _lib.NewsRecHIPError("gather_rows: idx must be contiguous int32")
    dim = src.shape[1]
    if out is None:
        out = torch.empty((n, dim), dtype=out_dtype or src.dtype, device=dev)
    _lib.call("nr_gather_rows", _dt(src, "src"), _dt(out, "out"), n, dim, _ptr(src), _rowmajor(src, "src"), _ptr(idx),
              _ptr(out), _rowmajor(out, "out"), _stream(dev))
    return out


def transpose(src: torch.Tensor, out_dtype: Optional[torch.dtype] = None,
              out: Optional[torch.Tensor] = None) -> torch.Tensor:
    dev = _dev(src, out)
    rows, cols = src.shape
    if out is None:
        out = torch.empty((cols, rows), dtype=out_dtype or src.dtype, device=dev)
    _lib.call("nr_transpose", _dt(src, "src"), _dt(out, "out"), rows, cols, _ptr(src), _rowmajor(src, "src"),
              _ptr(out), _rowmajor(out, "out"), _stream(dev))
    return out


def final_pool_fwd(xp: torch.Tensor, off: torch.Tensor):
    dev = _dev(xp, off)
    n_seg = off.numel() - 1
    users = torch.empty((n_seg, 1024), dtype=torch.float32, device=dev)
    z = torch.empty_like(users)
    _lib.call("nr_final_pool_fwd", _dt(xp, "xp"), n_seg, _ptr(off), _ptr(xp), _rowmajor(xp, "xp"), _ptr(users),
              _ptr(z), _stream(dev))
    return users, z


def final_pool_bwd(xp: torch.Tensor, off: torch.Tensor, users: torch.Tensor, z: torch.Tensor, du: torch.Tensor,
                   dx: torch.Tensor, dw: torch.Tensor) -> None:
    dev = _dev(xp, off, users, z, du, dx, dw)
    _lib.call("nr_final_pool_bwd", _dt(xp, "xp"), off.numel() - 1, _ptr(off), dx.shape[0], _ptr(xp),
              _rowmajor(xp, "xp"), _ptr(users), _ptr(z), _ptr(du), _ptr(dx), _rowmajor(dx, "dx"), _ptr(dw),
              _rowmajor(dw, "dw"), _stream(dev))


def cosine_margin(users: torch.Tensor, E: torch.Tensor, pos: torch.Tensor, neg: torch.Tensor, margin: float,
                  loss: torch.Tensor, du: torch.Tensor, dE: torch.Tensor,
                  s_out: Optional[torch.Tensor] = None) -> None:
    dev = _dev(users, E, pos, neg, loss, du, dE, s_out)
    _lib.call("nr_cosine_margin", users.shape[0], _ptr(users), _ptr(E), _rowmajor(E, "E"), _ptr(pos), _ptr(neg),
              ctypes.c_float(margin), _ptr(s_out), _ptr(loss), _ptr(du), _ptr(dE), _stream(dev))


def scatter_add_rows(src: torch.Tensor, idx: torch.Tensor, dst: torch.Tensor) -> None:
    dev = _dev(src, idx, dst)
    _lib.call("nr_scatter_add_rows", _dt(src, "src"), idx.numel(), src.shape[1], _ptr(src), _rowmajor(src, "src"),
              _ptr(idx), _ptr(dst), _rowmajor(dst, "dst"), _stream(dev))


def col_sum(src: torch.Tensor, out: torch.Tensor) -> None:
    dev = _dev(src, out)
    _lib.call("nr_col_sum", _dt(src, "src"), src.shape[0], src.shape[1], _ptr(src), _rowmajor(src, "src"), _ptr(out),
              _stream(dev))


def ln_param_grad(x: torch.Tensor, row_idx: Optional[torch.Tensor], eps: float, dy: torch.Tensor,
                  dgamma: torch.Tensor, dbeta: torch.Tensor) -> None:
    dev = _dev(x, row_idx, dy, dgamma, dbeta)
    dt = {torch.float32: _lib.NR_F32, torch.bfloat16: _lib.NR_BF16, torch.float16: _lib.NR_F16}[x.dtype]
    n = row_idx.numel() if row_idx is not None else x.shape[0]
    _lib.call("nr_ln_param_grad", dt, n, x.shape[1], _ptr(x), _rowmajor(x, "x"), _ptr(row_idx), ctypes.c_float(eps),
              _ptr(dy), _rowmajor(dy, "dy"), _ptr(dgamma), _ptr(dbeta), _stream(dev))


def sumsq(x: torch.Tensor, out: torch.Tensor) -> None:
    dev = _dev(x, out)
    _lib.call("nr_sumsq", x.numel(), _ptr(x), _ptr(out), _stream(dev))


def adamw(p: torch.Tensor, g: torch.Tensor, m: torch.Tensor, v: torch.Tensor, step: int, lr: float,
          betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.01, max_norm: float = 0.0,
          sumsq_t: Optional[torch.Tensor] = None, p_bf16: Optional[torch.Tensor] = None) -> None:
    dev = _dev(p, g, m, v, sumsq_t, p_bf16)
    _lib.call("nr_adamw", p.numel(), _ptr(p), _ptr(g), _ptr(m), _ptr(v), _ptr(p_bf16), step, ctypes.c_float(lr),
              ctypes.c_float(betas[0]), ctypes.c_float(betas[1]), ctypes.c_float(eps), ctypes.c_float(weight_decay),
              ctypes.c_float(max_norm), _ptr(sumsq_t), _stream(dev))


def _f32(t: torch.Tensor, name: str) -> None:
    if t.dtype != torch.float32:
        raise _lib.NewsRecHIPError(f"{name}: the latent-attention training kernels take f32 (got {t.dtype})")


def layernorm_bwd(x: torch.Tensor, gamma: Optional[torch.Tensor], dy: torch.Tensor, eps: float = 1e-5,
                  residual: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Input gradient of LayerNorm(x; gamma) for upstream dy (+ residual grad), f32."""
    for t, n in ((x, "x"), (dy, "dy")):
        _f32(t, n)
    out = torch.empty_like(x) if out is None else out
    dev = _dev(x, gamma, dy, residual, out)
    _lib.call("nr_layernorm_bwd", x.shape[0], x.shape[1], _ptr(x), _rowmajor(x, "x"), _ptr(gamma),
              ctypes.c_float(eps), _ptr(dy), _rowmajor(dy, "dy"), _ptr(residual),
              _rowmajor(residual, "residual") if residual is not None else 0, _ptr(out), _rowmajor(out, "out"),
              _stream(dev))
    return out


def softmax64_bwd(p: torch.Tensor, dp: torch.Tensor, out_dtype: torch.dtype = torch.float32) -> torch.Tensor:
    """dS of a softmax over groups of 64 columns, from its output p and upstream dp
    (f32 inputs; dS f32 or bf16)."""
    _f32(p, "p")
    _f32(dp, "dp")
    out = torch.empty(p.shape, dtype=out_dtype, device=p.device)
    dev = _dev(p, dp, out)
    _lib.call("nr_softmax64_bwd", _dtype(out, "out"), p.shape[0], p.shape[1], _ptr(p), _rowmajor(p, "p"), _ptr(dp),
              _rowmajor(dp, "dp"), _ptr(out), _rowmajor(out, "out"), _stream(dev))
    return out


def geglu_fwd(g: torch.Tensor, out_dtype: torch.dtype = torch.float32) -> torch.Tensor:
    """a * gelu(gates) with a, gates = g.chunk(2, -1) (f32 in, exact erf; out f32 or bf16)."""
    _f32(g, "g")
    f = g.shape[1] // 2
    z = torch.empty((g.shape[0], f), dtype=out_dtype, device=g.device)
    dev = _dev(g, z)
    _lib.call("nr_geglu_fwd", _dtype(z, "z"), g.shape[0], f, _ptr(g), _rowmajor(g, "g"), _ptr(z), f, _stream(dev))
    return z


def geglu_bwd(g: torch.Tensor, dz: torch.Tensor, out_dtype: torch.dtype = torch.float32) -> torch.Tensor:
    _f32(g, "g")
    _f32(dz, "dz")
    f = g.shape[1] // 2
    dg = torch.empty(g.shape, dtype=out_dtype, device=g.device)
    dev = _dev(g, dz, dg)
    _lib.call("nr_geglu_bwd", _dtype(dg, "dg"), g.shape[0], f, _ptr(g), _rowmajor(g, "g"), _ptr(dz), _rowmajor(dz, "dz"),
              _ptr(dg), _rowmajor(dg, "dg"), _stream(dev))
    return dg
