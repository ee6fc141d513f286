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
the HIP path uses (drop_hash below = nr_common.h drop_hash), indexed by the
packed valid-slot row (CSR order) and the column, so both sides see the same
masks; p = 0 reproduces the reference exactly (tests/golden/train_step.npz).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def drop_hash(seed: int, idx: np.ndarray) -> np.ndarray:
    """splitmix64 finaliser of seed + (idx + 1) * golden, upper 32 bits (uint32)."""
    with np.errstate(over="ignore"):
        z = np.uint64(seed & 0xFFFFFFFFFFFFFFFF) + (idx.astype(np.uint64) + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return (z >> np.uint64(32)).astype(np.uint32)


def keep_mask(seed: int, rows: np.ndarray, ncols: int, p: float) -> torch.Tensor:
    """keep[r, c] for packed slot rows `rows`: drop iff hash < p * 2^32."""
    thr = min(int(p * 4294967296.0), 0xFFFFFFFF)
    idx = rows.astype(np.uint64)[:, None] * np.uint64(ncols) + np.arange(ncols, dtype=np.uint64)[None, :]
    return torch.from_numpy((drop_hash(seed, idx) >= np.uint32(thr)).astype(np.float32))


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


def _loss(P, tok_last, hist_groups, pos, neg, p, seeds, ln_eps, margin, pooler="final"):
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
        out = pool_ref.latent_attention_forward({k[7:]: v for k, v in P.items() if k.startswith("latent.")},
                                                second, mask)
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
                margin=2.0):
    """The train_one_epoch loop (trainer.py:1044-1069: zero_grad, forward, loss,
    backward, clip_grad_norm_, AdamW.step with ONE persistent optimizer) over
    `batches` = list of (tok_last, hist_groups, pos, neg), dropout off, with
    FinalAttention (params "ln.*", "linear*") or the latent pooler (params
    "ln.*", "latent.<LatentAttentionModel name>").  Returns (per-step losses,
    per-step clipped-grad total norms, params after)."""
    P = _leaf(params)
    plist = list(P.values())
    opt = torch.optim.AdamW(plist, lr=lr, weight_decay=weight_decay)
    losses, norms = [], []
    for tok_last, groups, pos, neg in batches:
        opt.zero_grad()
        loss = _loss(P, tok_last, groups, pos, neg, 0.0, (0, 0, 0), ln_eps, margin, pooler)
        loss.backward()
        norms.append(float(torch.nn.utils.clip_grad_norm_(plist, max_norm=max_norm)))
        opt.step()
        losses.append(float(loss.detach()))
    return losses, norms, {k: v.detach().clone() for k, v in P.items()}
