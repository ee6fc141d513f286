"""ORACLE (test infrastructure only): token-attention encoder + last_token_pool.

Restates FirstAttentionPoolFunc(last_token_pool) (modeling_utils.py:498-524)
on the CPU in fp32:
  MyEncoder.forward  attention.py:204-207  loop over layers
  MyLayer.forward    attention.py:174-194  returns g_mlp_layernorm(hidden_states)
                     (:193 overwrites the attention result; eps 1e-12 :155)
  last_token_pool    modeling_utils.py:37-48  [:, -1] if every row's last mask
                     slot is set, else index mask.sum(1) - 1 (torch wraps -1)
and the sqlite path of apply_token_attn (data_model_helper.py:390-413) with
token_attention_eval_collate_fn / get_embeds_from_db (data_utils.py:878-933).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def encoder_forward(sd: dict, x: torch.Tensor, num_layers: int = 1, eps: float = 1e-12) -> torch.Tensor:
    for i in range(num_layers):
        p = f"encoder.layer.{i}.g_mlp_layernorm."
        x = F.layer_norm(x, (x.shape[-1],), sd[p + "weight"], sd[p + "bias"], eps)
    return x


def last_token_pool(h: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
    if int(mask[:, -1].sum()) == mask.shape[0]:
        return h[:, -1]
    return h[torch.arange(h.shape[0]), mask.sum(dim=1) - 1]


def first_attention_pool(sd: dict, emb: torch.Tensor, mask: torch.Tensor, num_layers: int = 1) -> torch.Tensor:
    return last_token_pool(encoder_forward(sd, emb.float(), num_layers), mask)


def apply_token_attn(sd: dict, states, batch: int = 3) -> torch.Tensor:
    """states: list of per-news [L_i, D] tensors in id order."""
    out = []
    for a in range(0, len(states), batch):
        group = states[a:a + batch]
        width = max(len(t) for t in group)
        emb = torch.zeros((len(group), width, group[0].shape[1]))
        mask = torch.zeros((len(group), width), dtype=torch.int32)
        for r, t in enumerate(group):
            emb[r, :len(t)] = t.float()
            mask[r, :len(t)] = 1
        out.append(first_attention_pool(sd, emb, mask))
    return torch.cat(out)
