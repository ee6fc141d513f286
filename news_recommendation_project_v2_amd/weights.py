"""Deterministic, portable weight and table generator.

The reference ships no checkpoints; the pooler checkpoints
``models/final_attn/Epoch_5.pt`` that ``scripts/eval.py:68-70`` loads do not
exist anywhere.  Parity fixtures, tests and the benchmark therefore use weights
produced by this generator, which is pure integer arithmetic (splitmix64) so
the same (seed, tensor name) gives bit-identical float32 tensors in this
container, on the GPU box and in the golden-vector script.

Element ``i`` of tensor ``name`` under ``seed``::

    key  = splitmix64(seed ^ fnv1a64(name))
    z_i  = splitmix64_mix(key + (i + 1) * GOLDEN)
    u_i  = (z_i >> 11) * 2**-53                      in [0, 1)

Linear weights/biases are ``(2u - 1) * 1/sqrt(fan_in)`` (PyTorch's default
``nn.Linear`` bound), LayerNorm is gamma=1, beta=0 (PyTorch default), latents
and news tables are N(0, 1) by Box-Muller over two streams.
"""
from __future__ import annotations

import math
from typing import Dict

import numpy as np
import torch

GENERATOR_VERSION = 1

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def _fnv1a64(s: str) -> int:
    h = 0xCBF29CE484222325
    for b in s.encode():
        h ^= b
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


def _mix(z: np.ndarray) -> np.ndarray:
    z = (z ^ (z >> np.uint64(30))) * _M1
    z = (z ^ (z >> np.uint64(27))) * _M2
    return z ^ (z >> np.uint64(31))


def _key(seed: int, name: str) -> np.uint64:
    k = np.array([(seed ^ _fnv1a64(name)) & 0xFFFFFFFFFFFFFFFF], dtype=np.uint64)
    return _mix(k + _GOLDEN)[0]


def uniform01(seed: int, name: str, n: int) -> np.ndarray:
    """float64 uniforms in [0, 1) for tensor ``name`` (n elements)."""
    key = _key(seed, name)
    out = np.empty(n, dtype=np.float64)
    chunk = 1 << 22
    with np.errstate(over="ignore"):
        for s in range(0, n, chunk):
            e = min(n, s + chunk)
            idx = np.arange(s + 1, e + 1, dtype=np.uint64)
            z = _mix(key + idx * _GOLDEN)
            out[s:e] = (z >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)
    return out


def uniform_tensor(seed: int, name: str, shape, bound: float) -> torch.Tensor:
    n = int(np.prod(shape))
    u = uniform01(seed, name, n)
    v = ((2.0 * u - 1.0) * bound).astype(np.float32)
    return torch.from_numpy(v.reshape(shape))


def normal_tensor(seed: int, name: str, shape) -> torch.Tensor:
    n = int(np.prod(shape))
    u1 = uniform01(seed, name + "#bm1", n)
    u2 = uniform01(seed, name + "#bm2", n)
    r = np.sqrt(-2.0 * np.log1p(-u1))  # 1-u1 in (0, 1]
    v = (r * np.cos(2.0 * math.pi * u2)).astype(np.float32)
    return torch.from_numpy(v.reshape(shape))


def linear_params(seed: int, prefix: str, out_f: int, in_f: int, bias: bool = True) -> Dict[str, torch.Tensor]:
    bound = 1.0 / math.sqrt(in_f)
    d = {prefix + "weight": uniform_tensor(seed, prefix + "weight", (out_f, in_f), bound)}
    if bias:
        d[prefix + "bias"] = uniform_tensor(seed, prefix + "bias", (out_f,), bound)
    return d


def final_attention_state_dict(seed: int = 1234, reduced_dim: int = 1024, hidden_dim: int = 4096) -> Dict[str, torch.Tensor]:
    """State dict with the reference ``FinalAttention`` keys
    (modeling_utils.py:185-192)."""
    sd: Dict[str, torch.Tensor] = {}
    sd.update(linear_params(seed, "linear1.", hidden_dim, reduced_dim))
    sd.update(linear_params(seed, "linear2.", hidden_dim, hidden_dim))
    sd.update(linear_params(seed, "linear3.", reduced_dim, hidden_dim))
    sd.update(linear_params(seed, "linear4.", hidden_dim, reduced_dim))
    sd.update(linear_params(seed, "linear5.", reduced_dim, hidden_dim, bias=False))
    return sd


def latent_attention_state_dict(seed: int = 1234, dim: int = 1024, num_latents: int = 64,
                                heads: int = 8, dim_head: int = 512, ff_mult: int = 4,
                                ln_random: bool = False) -> Dict[str, torch.Tensor]:
    """State dict with the reference ``LatentAttentionModel`` keys
    (latent_attention.py:115-131).  ``ln_random`` perturbs the LayerNorm
    affine parameters (tests use it so gamma/beta are exercised)."""
    inner = heads * dim_head
    sd: Dict[str, torch.Tensor] = {}
    sd["latents"] = normal_tensor(seed, "latents", (num_latents, dim))
    p = "cross_attend_blocks.0."
    sd.update(linear_params(seed, p + "fn.to_q.", inner, dim, bias=False))
    sd.update(linear_params(seed, p + "fn.to_kv.", 2 * inner, dim, bias=False))
    sd.update(linear_params(seed, p + "fn.to_out.", dim, inner, bias=False))
    for ln in (p + "norm.", p + "norm_context.", "cross_attend_blocks.1.norm."):
        if ln_random:
            sd[ln + "weight"] = 1.0 + uniform_tensor(seed, ln + "weight", (dim,), 0.25)
            sd[ln + "bias"] = uniform_tensor(seed, ln + "bias", (dim,), 0.25)
        else:
            sd[ln + "weight"] = torch.ones(dim)
            sd[ln + "bias"] = torch.zeros(dim)
    q = "cross_attend_blocks.1.fn.net."
    sd.update(linear_params(seed, q + "0.", dim * ff_mult * 2, dim))
    sd.update(linear_params(seed, q + "2.", dim, dim * ff_mult))
    # order keys like the reference module's state_dict()
    order = ["latents",
             p + "fn.to_q.weight", p + "fn.to_kv.weight", p + "fn.to_out.weight",
             p + "norm.weight", p + "norm.bias", p + "norm_context.weight", p + "norm_context.bias",
             q + "0.weight", q + "0.bias", q + "2.weight", q + "2.bias",
             "cross_attend_blocks.1.norm.weight", "cross_attend_blocks.1.norm.bias"]
    return {k: sd[k] for k in order}


def xlmr_state_dict(seed: int = 1234, n_layers: int = 24, vocab: int = 250002, hidden: int = 1024,
                    ffn: int = 4096, max_pos: int = 514) -> Dict[str, torch.Tensor]:
    """transformers XLMRobertaModel keys (encoder part; the unused CLS pooler is
    omitted).  Linear layers use the nn.Linear bound; embeddings U(-0.05, 0.05);
    LayerNorms gamma = 1 + U(-0.1, 0.1), beta = U(-0.02, 0.02) so they are exercised."""
    sd: Dict[str, torch.Tensor] = {}
    e = "embeddings."
    sd[e + "word_embeddings.weight"] = uniform_tensor(seed, e + "word", (vocab, hidden), 0.05)
    sd[e + "position_embeddings.weight"] = uniform_tensor(seed, e + "pos", (max_pos, hidden), 0.05)
    sd[e + "token_type_embeddings.weight"] = uniform_tensor(seed, e + "type", (1, hidden), 0.05)

    def ln(prefix):
        sd[prefix + "weight"] = 1.0 + uniform_tensor(seed, prefix + "weight", (hidden,), 0.1)
        sd[prefix + "bias"] = uniform_tensor(seed, prefix + "bias", (hidden,), 0.02)

    ln(e + "LayerNorm.")
    for i in range(n_layers):
        p = f"encoder.layer.{i}."
        for nm in ("query", "key", "value"):
            sd.update(linear_params(seed, p + f"attention.self.{nm}.", hidden, hidden))
        sd.update(linear_params(seed, p + "attention.output.dense.", hidden, hidden))
        ln(p + "attention.output.LayerNorm.")
        sd.update(linear_params(seed, p + "intermediate.dense.", ffn, hidden))
        sd.update(linear_params(seed, p + "output.dense.", hidden, ffn))
        ln(p + "output.LayerNorm.")
    return sd


def token_attn_state_dict(seed: int = 1234, hidden: int = 1024, num_layers: int = 1, heads: int = 8,
                          intermediate: int = 3072) -> Dict[str, torch.Tensor]:
    """State dict with the reference ``FirstAttentionPoolFunc`` keys
    (modeling_utils.py:498-513 -> attention.py:28-207): ``encoder.layer.{i}.``
    attention.qkv_proj / o_proj, g_mlp.up_gate_proj / down_proj, and the two
    LayerNorms (gamma = 1 + U(-0.25, 0.25), beta = U(-0.25, 0.25) so they are
    exercised)."""
    sd: Dict[str, torch.Tensor] = {}
    for i in range(num_layers):
        p = f"encoder.layer.{i}."
        sd.update(linear_params(seed, p + "attention.qkv_proj.", 3 * hidden, hidden))
        sd.update(linear_params(seed, p + "attention.o_proj.", hidden, hidden))
        sd.update(linear_params(seed, p + "g_mlp.up_gate_proj.", 2 * intermediate, hidden, bias=False))
        sd.update(linear_params(seed, p + "g_mlp.down_proj.", hidden, intermediate))
        for ln in ("attn_layernorm.", "g_mlp_layernorm."):
            sd[p + ln + "weight"] = 1.0 + uniform_tensor(seed, p + ln + "weight", (hidden,), 0.25)
            sd[p + ln + "bias"] = uniform_tensor(seed, p + ln + "bias", (hidden,), 0.25)
    return sd


def news_table(seed: int, n: int, dim: int = 1024, name: str = "news_table") -> torch.Tensor:
    """Synthetic news-embedding table: N(0,1) rows, matching the statistics of
    the LayerNorm-output ``new_embeddings/`` that eval.py loads."""
    return normal_tensor(seed, name, (n, dim))
