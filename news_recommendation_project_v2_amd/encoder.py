"""Title encoder on the MI355X path.

Replaces, for the e5-large-instruct / XLM-R-large encoder that
``get_embeddings`` (data_model_helper.py:45-84) runs through
``get_embed_from_model`` / ``get_text_embed_eval`` (modeling_utils.py:282-323):
  * padded batches of tokenised titles, the full HF forward, the D2H copy of
    every [B, L, 1024] hidden state and ``average_pool`` + ``F.normalize`` on
    the host,
with packed varlen token rows on the device (no padding) and ONE C-ABI call
per chunk, ``nr_encoder_forward``: embedding + LN, per layer a fused QKV GEMM,
the MFMA varlen attention kernel, GEMMs with residual / GELU epilogues,
post-LayerNorms, and the masked mean (average_pool; + F.normalize only for
the e5-instruct branch of get_embeddings) by the segmented pool kernel over
consecutive token rows.  Only the [B, 1024] embeddings leave the device.

Weights use the transformers ``XLMRobertaModel`` state-dict keys
(``embeddings.*``, ``encoder.layer.{i}.*``; a ``roberta.``/``model.`` prefix is
stripped), loaded with ``torch.load(weights_only=True)`` or safetensors.
"""
from __future__ import annotations

import math
from pathlib import Path
from typing import Iterable, Optional, Sequence

import numpy as np
import torch

from . import _lib, ops
from .config import NEWS_TEXT_MAXLEN

PAD_ID = 1          # XLM-R <pad>; positions start at PAD_ID + 1
LN_EPS = 1e-5       # XLM-R layer_norm_eps (NOT XLMRobertaConfig's 1e-12 default)
HIDDEN = 1024
HEADS = 16
FFN = 4096


def strip_prefix(sd: dict) -> dict:
    out = {}
    for k, v in sd.items():
        for p in ("roberta.", "model.", "xlm_roberta."):
            if k.startswith(p):
                k = k[len(p):]
        out[k] = v
    return out


def positions_for(ids: np.ndarray, lens: np.ndarray) -> np.ndarray:
    """HF create_position_ids_from_input_ids per packed sequence:
    pad + cumsum(id != pad) * (id != pad)."""
    m = (np.asarray(ids) != PAD_ID).astype(np.int64)
    lens = np.asarray(lens, dtype=np.int64)
    starts = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    cs = np.cumsum(m)
    before = np.where(starts > 0, cs[np.maximum(starts - 1, 0)], 0)  # non-pad count before each sequence
    return ((cs - np.repeat(before, lens)) * m + PAD_ID).astype(np.int32)


class XLMREncoder:
    # max_tokens: tokens per nr_encoder_forward call.  The workspace is ~14 KB
    # per bf16 token (QKV / FFN hidden [T x 4096] + three [T x 1024]): 1 M
    # tokens = 15 GB of the MI355X's 288 GB, so a 16 k-title query pass (~750 k
    # tokens) is one call and its GEMMs run as few, full-size persistent launches.
    def __init__(self, state_dict: dict, dtype: torch.dtype = torch.float32, device=None,
                 max_tokens: int = 1 << 20):
        sd = strip_prefix(state_dict)
        self.dtype = dtype
        self.device = device or torch.device("cuda")
        self.max_tokens = max_tokens
        n = 0
        while f"encoder.layer.{n}.attention.self.query.weight" in sd:
            n += 1
        self.n_layers = n
        dev, dt = self.device, dtype
        w = lambda k: sd[k].to(dev, dt).contiguous()
        f = lambda k: sd[k].to(dev, torch.float32).contiguous()
        self.word = w("embeddings.word_embeddings.weight")
        self.pos = w("embeddings.position_embeddings.weight")
        self.type0 = w("embeddings.token_type_embeddings.weight")[0].contiguous()
        self.eln = (f("embeddings.LayerNorm.weight"), f("embeddings.LayerNorm.bias"))
        self.layers = []
        for i in range(n):
            p = f"encoder.layer.{i}."
            a = p + "attention."
            wqkv = torch.cat([sd[a + "self.query.weight"], sd[a + "self.key.weight"], sd[a + "self.value.weight"]])
            bqkv = torch.cat([sd[a + "self.query.bias"], sd[a + "self.key.bias"], sd[a + "self.value.bias"]])
            self.layers.append({
                "wqkv": wqkv.to(dev, dt).contiguous(), "bqkv": bqkv.to(dev, torch.float32).contiguous(),
                "wo": w(a + "output.dense.weight"), "bo": f(a + "output.dense.bias"),
                "ln1": (f(a + "output.LayerNorm.weight"), f(a + "output.LayerNorm.bias")),
                "w1": w(p + "intermediate.dense.weight"), "b1": f(p + "intermediate.dense.bias"),
                "w2": w(p + "output.dense.weight"), "b2": f(p + "output.dense.bias"),
                "ln2": (f(p + "output.LayerNorm.weight"), f(p + "output.LayerNorm.bias")),
            })

        self._emb = {"word": self.word, "pos": self.pos, "type": self.type0, "ln_g": self.eln[0], "ln_b": self.eln[1]}
        self._layers = (_lib.EncoderLayer * n)()
        for i, L in enumerate(self.layers):
            ptrs = [L["wqkv"], L["bqkv"], L["wo"], L["bo"], L["ln1"][0], L["ln1"][1], L["w1"], L["b1"], L["w2"],
                    L["b2"], L["ln2"][0], L["ln2"][1]]
            for (name, _), t in zip(_lib.EncoderLayer._fields_, ptrs):
                setattr(self._layers[i], name, t.data_ptr())
        self._ws = None

    @classmethod
    def from_pretrained_dir(cls, path, **kw) -> "XLMREncoder":
        """Local HF directory (model.safetensors or pytorch_model.bin); no network."""
        path = Path(path)
        st = path / "model.safetensors"
        if st.is_file():
            from safetensors.torch import load_file
            sd = load_file(str(st))
        else:
            sd = torch.load(path / "pytorch_model.bin", weights_only=True, map_location="cpu")
        return cls(sd, **kw)

    # ------------------------------------------------------------------ forward
    def _forward(self, ids: np.ndarray, lens: np.ndarray, pool: Optional[str], want_hidden: bool,
                 status: torch.Tensor):
        """One nr_encoder_forward call over a chunk of packed sequences."""
        dev = self.device
        ids_d = torch.as_tensor(np.ascontiguousarray(ids, dtype=np.int32)).to(dev)
        lens_d = torch.as_tensor(np.ascontiguousarray(lens, dtype=np.int32)).to(dev)
        T = int(np.asarray(lens, dtype=np.int64).sum())
        need = _lib.load().nr_encoder_workspace_bytes(_lib.NR_F32 if self.dtype == torch.float32 else _lib.NR_BF16,
                                                      T, len(lens))
        if self._ws is None or self._ws.numel() < need:
            self._ws = torch.empty(need, dtype=torch.uint8, device=dev)
        return ops.encoder_forward(self._layers, self._emb, ids_d, lens_d, T, pool=pool, want_hidden=want_hidden,
                                   eps=LN_EPS, workspace=self._ws, status=status)

    @staticmethod
    def _check_status(status: torch.Tensor) -> None:
        st = int(status.item())
        if st & 2:  # the reference's nn.Embedding lookup raises IndexError here
            raise IndexError("token id outside the encoder vocabulary")
        if st & 1:
            raise IndexError(f"sequence longer than the position table ({NEWS_TEXT_MAXLEN} tokens after truncation)")

    def _chunks(self, lens: np.ndarray):
        """Consecutive sequence ranges [s, e) of at most max_tokens tokens."""
        off = np.concatenate([[0], np.cumsum(lens)])
        n, s = len(lens), 0
        while s < n:
            # the last e with off[e] - off[s] <= max_tokens (at least one sequence):
            # one binary search, not a Python step per sequence (16 k titles per pass)
            e = int(np.searchsorted(off, off[s] + self.max_tokens, side="right")) - 1
            e = min(max(e, s + 1), n)
            yield s, e, off
            s = e

    def encode_packed(self, ids: np.ndarray, lens: np.ndarray, normalize: bool = False) -> torch.Tensor:
        """ids: flat int tokens of all sequences; lens: tokens per sequence.
        Returns average_pool(last_hidden_state) [B, 1024] f32 on the device
        (get_text_embed_eval, modeling_utils.py:282-300), L2-normalised when
        ``normalize`` (the e5-instruct branch of get_embeddings,
        data_model_helper.py:65-78)."""
        ids = np.asarray(ids)
        lens = np.asarray(lens, dtype=np.int64)
        if np.any(lens <= 0):
            raise ValueError("every sequence needs at least one token")
        status = torch.zeros(1, dtype=torch.int32, device=self.device)
        pool = "normalize" if normalize else "mean"
        out = [self._forward(ids[off[s]:off[e]], lens[s:e], pool, False, status)[0] for s, e, off in self._chunks(lens)]
        self._check_status(status)
        return torch.cat(out) if out else torch.zeros((0, HIDDEN), device=self.device)

    def hidden_states_packed(self, ids: np.ndarray, lens: np.ndarray):
        """Per-token last_hidden_state of every sequence (the tensors the reference
        stores per news in its sqlite token DB, modeling_utils.py:456-478).
        Yields (first sequence index, packed rows [T, 1024] on device, lengths)."""
        ids = np.asarray(ids)
        lens = np.asarray(lens, dtype=np.int64)
        if np.any(lens <= 0):
            raise ValueError("every sequence needs at least one token")
        status = torch.zeros(1, dtype=torch.int32, device=self.device)
        for s, e, off in self._chunks(lens):
            _, x = self._forward(ids[off[s]:off[e]], lens[s:e], None, True, status)
            self._check_status(status)
            yield s, x, lens[s:e]

    def encode_padded(self, input_ids: torch.Tensor, attention_mask: torch.Tensor) -> torch.Tensor:
        """Tokenizer-style right-padded batch -> embeddings (drops padded slots)."""
        m = attention_mask.bool().cpu().numpy()
        ids = input_ids.cpu().numpy()
        return self.encode_packed(ids[m], m.sum(1))


def tokenize(tokenizer, texts: Sequence[str], max_len: int) -> tuple[np.ndarray, np.ndarray]:
    """Tokenise to packed ids + lengths (eval_collate_fn data_utils.py:471-482
    without padding: truncation at max_len, special tokens added)."""
    enc = tokenizer(list(texts), max_length=max_len, truncation=True, padding=False)
    lens = np.array([len(x) for x in enc["input_ids"]], dtype=np.int64)
    ids = np.concatenate([np.asarray(x, dtype=np.int32) for x in enc["input_ids"]]) if len(lens) else np.zeros(0, np.int32)
    return ids, lens


def store_token_states(encoder: "XLMREncoder", ids: np.ndarray, lens: np.ndarray, db_name,
                       dtype: torch.dtype = torch.float16) -> int:
    """Write every sequence's per-token hidden states into the reference's
    sqlite token DB layout (store_text_embed_full_eval, modeling_utils.py:456-478):
    table ``tensors(id INTEGER PRIMARY KEY, data BLOB)``, ids 1.., each blob a
    ``torch.save`` of a [L_valid, 1024] tensor (fp16 like the reference's fp16
    model outputs).  Returns the number of rows written."""
    import io
    import sqlite3
    n = 0
    with sqlite3.connect(str(db_name)) as conn:
        conn.execute("DROP TABLE IF EXISTS tensors;")
        conn.execute("CREATE TABLE tensors (id INTEGER PRIMARY KEY, data BLOB)")
        for _, x, ln in encoder.hidden_states_packed(ids, lens):
            host = x.to(dtype).cpu()
            for t in torch.split(host, [int(v) for v in ln]):
                buf = io.BytesIO()
                torch.save(t.clone(), buf)
                conn.execute("INSERT INTO tensors (data) VALUES (?)", (buf.getvalue(),))
                n += 1
    return n


def get_embeddings(model_path: str, news_list: Iterable[str], news_text_dict: dict[str, str],
                   dtype: torch.dtype = torch.float32):
    """data_model_helper.get_embeddings (data_model_helper.py:45-84) for a LOCAL
    model directory: returns (query_embeds, passage_embeds) for e5-instruct
    models (query text = QUERY_INSTRUCTION + text), else passage embeds."""
    from transformers import AutoTokenizer

    from .config import NEWS_TEXT_MAXLEN, QUERY_INSTRUCTION
    tok = AutoTokenizer.from_pretrained(model_path)
    enc = XLMREncoder.from_pretrained_dir(model_path, dtype=dtype)
    news = list(news_list)
    passages = [news_text_dict[n] for n in news]
    if "e5" in str(model_path) and "instruct" in str(model_path):
        # data_model_helper.py:59-80: query + passage passes, each F.normalize'd
        q = enc.encode_packed(*tokenize(tok, [QUERY_INSTRUCTION + t for t in passages], NEWS_TEXT_MAXLEN),
                              normalize=True).cpu()
        p = enc.encode_packed(*tokenize(tok, passages, NEWS_TEXT_MAXLEN), normalize=True).cpu()
        return q, p
    # data_model_helper.py:81-84: any other model returns the raw average_pool
    return enc.encode_packed(*tokenize(tok, passages, NEWS_TEXT_MAXLEN)).cpu()
