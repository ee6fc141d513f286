"""ORACLE (test infrastructure only): one config-5 training step on the CPU.

Restates the body of AttentionAttentionTrainer.train_one_epoch
(trainer.py:1044-1069) with torch autograd in fp32:
  first_res  = token_model(tok, mask)          FirstAttentionPoolFunc = g_mlp_LN of
                                               the last valid token (attention.py:193,
                                               modeling_utils.py:37-48)
  second_res = first_res[hist] * hist_mask     trainer.py:1052-1054
  outputs    = FinalAttention(second_res, m)   modeling_utils.py:218-228, train mode
  res        = F.cosine_similarity(outputs.repeat(2, 1), first_res[pos ‖ neg])
  loss       = MarginRankingLoss(2)(*res.chunk(2), 1)
  backward; clip_grad_norm_(params, 0.5); AdamW(lr, wd 0.01).step()
Dropout (nn.Dropout p in the reference) is drawn from the counter-hash stream
the HIP path uses (drop_hash4 / keep_mask below = nr_common.h drop_at), indexed by the
packed valid-slot row (CSR order) and the column, so both sides see the same
masks; p = 0 reproduces the reference exactly (tests/golden/train_step.npz).
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def drop_hash4(seed: int, g: np.ndarray) -> np.ndarray:
    """splitmix64 finaliser of seed + (g + 1) * golden (uint64): the hash of
    dropout group g = 4 consecutive elements (nr_common.h drop_hash4)."""
    with np.errstate(over="ignore"):
        z = np.uint64(seed & 0xFFFFFFFFFFFFFFFF) + (g.astype(np.uint64) + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def dropout_threshold(p: float) -> int:
    """round(p * 2^16), clamped to [0, 65536] (nr_common.h dropout_threshold)."""
    return int(min(max(round(p * 65536.0), 0), 65536))


def keep_mask(seed: int, rows: np.ndarray, ncols: int, p: float) -> torch.Tensor:
    """keep[r, c] for packed slot rows `rows`: element idx = row * ncols + c is
    dropped iff 16-bit field idx & 3 of drop_hash4(seed, idx >> 2) < round(p * 2^16)."""
    thr = np.uint64(dropout_threshold(p))
    idx = rows.astype(np.uint64)[:, None] * np.uint64(ncols) + np.arange(ncols, dtype=np.uint64)[None, :]
    field = (drop_hash4(seed, idx >> np.uint64(2)) >> ((idx & np.uint64(3)) * np.uint64(16))) & np.uint64(0xFFFF)
    return torch.from_numpy((field >= thr).astype(np.float32))


def final_attention_train(sd, emb, mask, seeds, p, slot_rows):
    """FinalAttention.forward in train mode with hash dropout; emb [B, L, D], mask
    [B, L]; slot_rows [B, L] = packed row of each valid slot (-1 padding)."""
    valid = slot_rows >= 0
    rows = slot_rows[valid]

    def drop(x, seed):
        if p == 0:
            return x
        m = torch.ones(x.shape)
        m[torch.from_numpy(valid)] = keep_mask(seed, rows, x.shape[-1], p)
        return x * m / (1 - p)

    x = drop(F.relu(F.linear(emb, sd["linear1.weight"], sd["linear1.bias"])), seeds[0])
    x = drop(F.relu(F.linear(x, sd["linear2.weight"], sd["linear2.bias"])), seeds[1])
    x = F.linear(x, sd["linear3.weight"], sd["linear3.bias"])
    w = drop(F.relu(F.linear(x, sd["linear4.weight"], sd["linear4.bias"])), seeds[2])
    w = F.linear(w, sd["linear5.weight"])
    w = torch.exp(w) * mask.unsqueeze(-1)
    w = w / (w.sum(dim=1, keepdim=True) + 1e-10)
    return (x * w).sum(dim=1)


class _BF16(torch.autograd.Function):
    """Round to bf16 (RNE) in the forward; the incoming gradient rounded the same
    way in the backward (a bf16-stored activation and its bf16-stored gradient)."""

    @staticmethod
    def forward(ctx, x):
        return x.to(torch.bfloat16).float()

    @staticmethod
    def backward(ctx, g):
        return g.to(torch.bfloat16).float()


def _bf16_weight(w):
    """bf16 copy of an f32 master weight; the gradient reaches the master unrounded."""
    return w + (w.detach().to(torch.bfloat16).float() - w.detach())


class _Split(torch.autograd.Function):
    """hi + lo bf16 pair of an f32 value in the forward (the split-bf16 operand of
    a bf16x3 GEMM); the gradient rounded to bf16 in the backward."""

    @staticmethod
    def forward(ctx, x):
        hi = x.to(torch.bfloat16).float()
        return hi + (x - hi).to(torch.bfloat16).float()

    @staticmethod
    def backward(ctx, g):
        return g.to(torch.bfloat16).float()


def _split_weight(w):
    hi = w.detach().to(torch.bfloat16).float()
    return w + (hi + (w.detach() - hi).to(torch.bfloat16).float() - w.detach())


def final_attention_train_bf16x3(sd, emb, mask):
    """BF16x3 NUMERICS MODEL (not the reference): the precise-forward variant of the
    bf16 step -- every forward GEMM operand split into a hi + lo bf16 pair (f32 to
    16 mantissa bits; the A_lo W_lo product dropped is below that), the backward
    as the bf16 model (bf16 weights, activations and gradients)."""
    r, sp = _BF16.apply, _Split.apply
    Wf = {i: _split_weight(sd[f"linear{i}.weight"]) for i in range(1, 6)}
    x = F.relu(F.linear(sp(emb), Wf[1], sd["linear1.bias"]))
    x = F.relu(F.linear(sp(x), Wf[2], sd["linear2.bias"]))
    x = F.linear(sp(x), Wf[3], sd["linear3.bias"])
    w = F.relu(F.linear(sp(x), Wf[4], sd["linear4.bias"]))
    w = torch.exp(F.linear(sp(w), Wf[5])) * mask.unsqueeze(-1)
    w = w / (w.sum(dim=1, keepdim=True) + 1e-10)
    return (x * w).sum(dim=1)


def final_attention_train_bf16(sd, emb, mask):
    """BF16 NUMERICS MODEL (not the reference): FinalAttention.forward
    (modeling_utils.py:218-228) with the HIP bf16 step's rounding points --
    bf16 weights, every activation the step stores (S, X1, X2, X, Y, P) rounded
    to bf16 and so their gradients; products exact, sums in f32, pooling in f32.
    What an ideal RNE bf16 implementation of the step computes (dropout off)."""
    r = _BF16.apply
    W = {i: _bf16_weight(sd[f"linear{i}.weight"]) for i in range(1, 6)}
    x = r(F.relu(F.linear(r(emb), W[1], sd["linear1.bias"])))
    x = r(F.relu(F.linear(x, W[2], sd["linear2.bias"])))
    x = r(F.linear(x, W[3], sd["linear3.bias"]))
    w = r(F.relu(F.linear(x, W[4], sd["linear4.bias"])))
    w = r(torch.exp(F.linear(w, W[5]))) * mask.unsqueeze(-1)
    w = w / (w.sum(dim=1, keepdim=True) + 1e-10)
    return (x * w).sum(dim=1)


def latent_attention_train_bf16(sd, emb, mask, heads=8):
    """BF16 NUMERICS MODEL (not the reference) of the latent bf16 step
    (csrc/latent_train.hip): the K/V fold A_h = K_h Wq_h / sqrt(512), Bt_h^T =
    V_h Wo_h^T from bf16 LN_c(latents) and bf16 weights; per slot S, X = LN_q(E[hist]),
    P = softmax64(X A^T), H1 = P Bt^T + S, Y = LN_f(H1), G = Y W1^T + b1 stored bf16;
    per batch row m = bf16(mean GEGLU(G)) W2^T + b2 + mean(H1) (f32), u = normalize(m).
    Same math as latent_attention.py:134-171 (the last layer commuted with the mean)."""
    r = _BF16.apply
    p, q_ = "cross_attend_blocks.0.", "cross_attend_blocks.1."
    d = emb.shape[-1]
    latn = r(F.layer_norm(sd["latents"], (d,), sd[p + "norm_context.weight"], sd[p + "norm_context.bias"], 1e-5))
    kv = r(F.linear(latn, _bf16_weight(sd[p + "fn.to_kv.weight"])))          # [64, 8192]
    k, v = kv.chunk(2, dim=-1)                                                 # [64, 4096] each
    wq, wo = _bf16_weight(sd[p + "fn.to_q.weight"]), _bf16_weight(sd[p + "fn.to_out.weight"])
    dh = k.shape[1] // heads
    A = r(torch.cat([k[:, h * dh:(h + 1) * dh] @ wq[h * dh:(h + 1) * dh] for h in range(heads)]) / math.sqrt(dh))
    BtT = r(torch.cat([v[:, h * dh:(h + 1) * dh] @ wo[:, h * dh:(h + 1) * dh].T for h in range(heads)]))  # [512, 1024]
    m = mask.bool()
    e = emb[m]                                                                 # [Hs, d] valid slots, CSR order
    S = r(e)
    X = r(F.layer_norm(e, (d,), sd[p + "norm.weight"], sd[p + "norm.bias"], 1e-5))
    Pm = r(torch.softmax((X @ A.T).reshape(-1, heads, 64), dim=-1).reshape(-1, heads * 64))
    H1 = r(Pm @ BtT + S)
    Y = r(F.layer_norm(H1, (d,), sd[q_ + "norm.weight"], sd[q_ + "norm.bias"], 1e-5))
    G = r(F.linear(Y, _bf16_weight(sd[q_ + "fn.net.0.weight"]), sd[q_ + "fn.net.0.bias"]))
    a, g = G.chunk(2, dim=-1)
    Z = a * F.gelu(g)
    lens = m.sum(dim=1)
    seg = torch.repeat_interleave(torch.arange(len(lens)), lens)
    zbar = r(torch.zeros((len(lens), Z.shape[1])).index_add(0, seg, Z) / lens[:, None])
    h1bar = torch.zeros((len(lens), d)).index_add(0, seg, H1) / lens[:, None]
    out = F.linear(zbar, _bf16_weight(sd[q_ + "fn.net.2.weight"]), sd[q_ + "fn.net.2.bias"]) + h1bar
    return F.normalize(out, p=2, dim=-1)


def _loss(P, tok_last, hist_groups, pos, neg, p, seeds, ln_eps, margin, pooler="final", numerics="f32"):
    E = F.layer_norm(tok_last.float(), (tok_last.shape[1],), P["ln.weight"], P["ln.bias"], ln_eps)
    B = len(hist_groups)
    L = max(len(h) for h in hist_groups)
    idx = torch.zeros((B, L), dtype=torch.long)
    mask = torch.zeros((B, L), dtype=torch.int32)
    slot_rows = -np.ones((B, L), dtype=np.int64)
    r = 0
    for b, h in enumerate(hist_groups):
        idx[b, :len(h)] = torch.as_tensor(np.asarray(h, dtype=np.int64))
        mask[b, :len(h)] = 1
        slot_rows[b, :len(h)] = np.arange(r, r + len(h))
        r += len(h)
    second = E[idx] * mask.unsqueeze(-1)
    if pooler == "latent":  # LatentAttentionModel in FinalAttention's slot (no dropout in that module)
        from oracle import pool_ref
        lsd = {k[7:]: v for k, v in P.items() if k.startswith("latent.")}
        out = (latent_attention_train_bf16(lsd, second, mask) if numerics == "bf16" else
               pool_ref.latent_attention_forward(lsd, second, mask))
    elif numerics == "bf16":
        out = final_attention_train_bf16(P, second, mask)
    elif numerics == "bf16x3":
        out = final_attention_train_bf16x3(P, second, mask)
    else:
        out = final_attention_train(P, second, mask, seeds, p, slot_rows)
    pn = torch.as_tensor(np.concatenate([pos, neg]).astype(np.int64))
    res = F.cosine_similarity(out.repeat((2, 1)), E[pn])
    return torch.nn.MarginRankingLoss(margin)(*torch.chunk(res, 2), torch.tensor([1.0]))


def _leaf(params):
    return {k: v.detach().clone().float().requires_grad_(True) for k, v in params.items()}


def train_step(params: dict, tok_last: torch.Tensor, hist_groups, pos, neg, *, p=0.0, seeds=(0, 0, 0), lr=1e-6,
               max_norm=0.5, weight_decay=0.01, ln_eps=1e-12, margin=2.0, do_step=True):
    """params: {"ln.weight", "ln.bias", "linear{i}.weight", "linear{i}.bias"} f32 CPU.
    tok_last [U, D] (last valid token per unique news); hist_groups: list of int
    arrays (indices into U); pos/neg [B].  Returns dict(loss, grads, total_norm,
    params_after)."""
    P = _leaf(params)
    loss = _loss(P, tok_last, hist_groups, pos, neg, p, seeds, ln_eps, margin)
    loss.backward()
    plist = [v for v in P.values() if v.grad is not None]
    grads = {k: v.grad.detach().clone() for k, v in P.items() if v.grad is not None}
    total = torch.nn.utils.clip_grad_norm_(plist, max_norm=max_norm)
    after = None
    if do_step:
        torch.optim.AdamW(plist, lr=lr, weight_decay=weight_decay).step()
        after = {k: v.detach().clone() for k, v in P.items()}
    return {"loss": float(loss), "grads": grads, "total_norm": float(total), "params_after": after}


def train_epoch(params: dict, batches, *, lr=1e-6, max_norm=0.5, weight_decay=0.01, ln_eps=1e-12, margin=2.0):
    """One epoch with a persistent AdamW (dropout off): batches = list of
    (tok_last, hist_groups, pos, neg, n_rows).  Returns (row-weighted mean loss,
    params after)."""
    P = _leaf(params)
    plist = list(P.values())
    opt = torch.optim.AdamW(plist, lr=lr, weight_decay=weight_decay)
    tot, cnt = 0.0, 0
    for tok_last, groups, pos, neg, n in batches:
        opt.zero_grad()
        loss = _loss(P, tok_last, groups, pos, neg, 0.0, (0, 0, 0), ln_eps, margin)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(plist, max_norm=max_norm)
        opt.step()
        tot += float(loss) * n
        cnt += n
    return tot / cnt, {k: v.detach().clone() for k, v in P.items()}


def train_steps(params: dict, batches, *, pooler="final", lr=1e-6, max_norm=0.5, weight_decay=0.01, ln_eps=1e-12,
                margin=2.0, numerics="f32"):
    """The train_one_epoch loop (trainer.py:1044-1069: zero_grad, forward, loss,
    backward, clip_grad_norm_, AdamW.step with ONE persistent optimizer) over
    `batches` = list of (tok_last, hist_groups, pos, neg), dropout off, with
    FinalAttention (params "ln.*", "linear*") or the latent pooler (params
    "ln.*", "latent.<LatentAttentionModel name>").  numerics="bf16" (FinalAttention
    only): the bf16 numerics model above instead of f32 -- the drift an ideal bf16
    implementation shows against the f32 loop.  Returns (per-step losses,
    per-step clipped-grad total norms, params after)."""
    P = _leaf(params)
    plist = list(P.values())
    opt = torch.optim.AdamW(plist, lr=lr, weight_decay=weight_decay)
    losses, norms = [], []
    for tok_last, groups, pos, neg in batches:
        opt.zero_grad()
        loss = _loss(P, tok_last, groups, pos, neg, 0.0, (0, 0, 0), ln_eps, margin, pooler, numerics)
        loss.backward()
        norms.append(float(torch.nn.utils.clip_grad_norm_(plist, max_norm=max_norm)))
        opt.step()
        losses.append(float(loss.detach()))
    return losses, norms, {k: v.detach().clone() for k, v in P.items()}
