"""ORACLE (test infrastructure only): title encoder on the CPU.

The reference's encoder is third-party: transformers' XLMRobertaModel
(AutoModel of intfloat/multilingual-e5-large-instruct, modeling_utils.py:92-103;
transformers is unpinned in pyproject.toml:20, the installed 5.15.0 is used).
This restates the reference's use of it: padded batch forward, then
average_pool (modeling_utils.py:55-59) and F.normalize(p=2, dim=1)
(data_model_helper.py:65-78).  Weights come from weights.xlmr_state_dict.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F


def build_model(state_dict: dict, n_layers: int, vocab: int):
    from transformers import XLMRobertaConfig, XLMRobertaModel
    cfg = XLMRobertaConfig(vocab_size=vocab, hidden_size=1024, num_hidden_layers=n_layers, num_attention_heads=16,
                           intermediate_size=4096, max_position_embeddings=514, layer_norm_eps=1e-5,
                           type_vocab_size=1, pad_token_id=1, hidden_act="gelu")
    m = XLMRobertaModel(cfg, add_pooling_layer=False)
    m.load_state_dict(state_dict, strict=False)
    return m.eval()


def encode(model, ids: np.ndarray, lens: np.ndarray, batch: int = 16) -> torch.Tensor:
    seqs, s = [], 0
    for L in lens:
        seqs.append(ids[s:s + L])
        s += L
    out = []
    with torch.no_grad():
        for b in range(0, len(seqs), batch):
            chunk = seqs[b:b + batch]
            width = max(len(x) for x in chunk)
            x = torch.ones((len(chunk), width), dtype=torch.long)
            m = torch.zeros((len(chunk), width), dtype=torch.long)
            for i, q in enumerate(chunk):
                x[i, :len(q)] = torch.as_tensor(q, dtype=torch.long)
                m[i, :len(q)] = 1
            h = model(input_ids=x, attention_mask=m).last_hidden_state
            h = h.masked_fill(~m[..., None].bool(), 0.0)
            out.append(h.sum(dim=1) / m.sum(dim=1)[..., None])
    return F.normalize(torch.cat(out), p=2, dim=1)
