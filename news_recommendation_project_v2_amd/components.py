"""Pipeline components of the hot path (reference components.py).

Kept: TransformData (45-114), EmbeddingsComponent (117-175),
SaveEmbeddingComponent (178-223), LoadEmbeddingComponent (226-258),
TokenEmbeddingsComponent (955-977), FinalAttentionComponent (980-1027,
transform only), StoreEmbeddingsComponent (858-880),
AttentionAttentionComponent (883-952, config-5 training), plus
LatentAttentionComponent — the same scoring with the latent pooler, which the
reference can only reach through get_latent_attention_model
(modeling_utils.py:151-155).  The other experiments' components and the Azure
upload are out of scope.
"""
from __future__ import annotations

from pathlib import Path
from typing import Any, Optional

import numpy as np
import torch

from .data_model_helper import apply_token_attn, get_embeddings, get_final_second_attention_score, store_embeddings
from .data_utils import split_impressions_and_history
from .modeling_utils import get_final_attention_model, get_latent_attention_model, get_token_attn_model
from .pipeline import PipelineComponent, check_req_keys


class TransformData(PipelineComponent):
    """Behaviours -> index arrays + per-news feature tensors (components.py:45-114).

    The reference requires the entity/category keys too; they are optional here
    because nothing on the embed -> pool -> score path reads them (their
    tensors are produced when present).
    """

    required_keys = {"behaviors"}

    def transform(self, context_dict: dict[str, Any]) -> dict[str, Any]:
        check_req_keys(self.required_keys, context_dict)
        behaviors = context_dict["behaviors"]
        new = context_dict.copy()
        new["ImpressionID"] = behaviors["ImpressionID"]
        new.update(split_impressions_and_history(behaviors["Impressions"], behaviors["History"]))
        new["history_bool"] = behaviors["History"].notna()
        news_list = new["news_list"]
        for src, dst in (("news_title_entity", "title_entity_embed"),
                         ("news_abstract_entity", "abstract_entity_embed")):
            if src in context_dict:
                new[dst] = torch.stack([torch.tensor(context_dict[src][i], dtype=torch.float32) for i in news_list])
                new.pop(src)
        for src, dst in (("news_category", "cat_indices"), ("news_subcategory", "subcat_indices")):
            if src in context_dict:
                new[dst] = torch.tensor([context_dict[src][i] for i in news_list], dtype=torch.int32).unsqueeze(-1)
                new.pop(src)
        new.pop("behaviors")
        return new


class EmbeddingsComponent(PipelineComponent):
    """Title encoder over news_list (components.py:117-175)."""

    required_keys = {"news_list", "news_text_dict"}

    def __init__(self, model_path: str):
        self.model_path = model_path

    def transform(self, context_dict):
        check_req_keys(self.required_keys, context_dict)
        new = context_dict.copy()
        emb = get_embeddings(self.model_path, new["news_list"], new["news_text_dict"])
        if isinstance(emb, tuple):
            new["query_news_embeddings"], new["news_embeddings"] = emb
        else:
            new["news_embeddings"] = emb
        return new


class SaveEmbeddingComponent(PipelineComponent):
    """torch.save tables as {save_dir}/{split}.pt (+ query_ prefix) (components.py:193-223)."""

    required_keys = {"news_embeddings", "news_dataset"}

    def __init__(self, save_dir: Path):
        self.save_dir = Path(save_dir)

    def transform(self, context_dict):
        check_req_keys(self.required_keys, context_dict)
        self.save_dir.mkdir(parents=True, exist_ok=True)
        name = context_dict["news_dataset"].value
        torch.save(context_dict["news_embeddings"], self.save_dir / f"{name}.pt")
        if "query_news_embeddings" in context_dict:
            torch.save(context_dict["query_news_embeddings"], self.save_dir / f"query_{name}.pt")
        return context_dict


class LoadEmbeddingComponent(PipelineComponent):
    """torch.load(weights_only=True) of the tables (components.py:234-258)."""

    required_keys = {"news_dataset"}

    def __init__(self, save_dir: Path):
        self.save_dir = Path(save_dir)

    def transform(self, context_dict):
        check_req_keys(self.required_keys, context_dict)
        name = context_dict["news_dataset"].value
        context_dict["news_embeddings"] = torch.load(self.save_dir / f"{name}.pt", weights_only=True)
        q = self.save_dir / f"query_{name}.pt"
        if q.exists():
            context_dict["query_news_embeddings"] = torch.load(q, weights_only=True)
        return context_dict


class StoreEmbeddingsComponent(PipelineComponent):
    """Per-token title hidden states -> sqlite token DB (components.py:858-880)."""

    required_keys = {"news_list", "news_text_dict"}

    def __init__(self, model_path: str, db_name: str):
        self.model_path = model_path
        self.db_name = db_name

    def transform(self, context_dict):
        check_req_keys(self.required_keys, context_dict)
        new = context_dict.copy()
        store_embeddings(self.model_path, new["news_list"], new["news_text_dict"], self.db_name)
        del new["news_text_dict"]
        return new


class AttentionAttentionComponent(PipelineComponent):
    """Config-5 training of the token-attention model + FinalAttention
    (components.py:883-952): ``train`` builds an AttentionAttentionTrainer on the
    impressions that have a history and runs ``num_epochs``; ``transform`` is the
    identity.  ``pooler="latent"`` trains LatentAttentionModel in FinalAttention's
    slot.  Extra keyword arguments (batch_size, dtype, lr, dropout, seed) go
    to the trainer."""

    required_keys = {"impression_rev_ind_array", "impression_len_list", "history_rev_ind_array",
                     "history_len_list", "history_bool"}
    train_required_keys = required_keys | {"labels"}

    def __init__(self, db_name: str, token_attention_model_path: Optional[Path] = None,
                 final_attention_model_path: Optional[Path] = None, log_dir: Optional[Path] = None,
                 token_ckpt_dir: Optional[Path] = None, final_attn_ckpt_dir: Optional[Path] = None, num_epochs=5,
                 exp_name: str = "", max_neg_ratio: Optional[float] = None, max_pos_ratio: Optional[float] = None,
                 rng=None, pooler: str = "final", **trainer_kw):
        self.db_name = db_name
        self.token_attention = get_token_attn_model(token_attention_model_path)
        if pooler not in ("final", "latent"):
            raise ValueError(f"AttentionAttentionComponent: pooler must be 'final' or 'latent', got {pooler!r}")
        # pooler="latent": BASELINE configs[4]'s pairing (token encoder + LatentAttentionModel)
        self.final_attention = (get_latent_attention_model(final_attention_model_path) if pooler == "latent" else
                                get_final_attention_model(final_attention_model_path))
        self.num_epochs = num_epochs
        self.exp_name = exp_name
        self.rng = rng if rng is not None else np.random.default_rng(1234)
        self.log_dir = log_dir
        self.token_ckpt_dir = token_ckpt_dir
        self.final_attn_ckpt_dir = final_attn_ckpt_dir
        self.max_neg_ratio = max_neg_ratio
        self.max_pos_ratio = max_pos_ratio
        self.trainer_kw = trainer_kw
        self.trainer = None

    def transform(self, context_dict):
        return context_dict

    def train(self, context_dict, val_context_dict=None):
        from .trainer import AttentionAttentionTrainer
        check_req_keys(self.train_required_keys, context_dict)
        hb = np.asarray(context_dict["history_bool"], dtype=bool)
        imp_len = np.asarray(context_dict["impression_len_list"])
        self.trainer = AttentionAttentionTrainer(
            db_name=self.db_name, token_attention_model=self.token_attention,
            final_attention_model=self.final_attention,
            train_history_rev_index=context_dict["history_rev_ind_array"][0],
            train_history_len_list=context_dict["history_len_list"],
            train_news_rev_index=context_dict["impression_rev_ind_array"][0][np.repeat(hb, imp_len)],
            train_impression_len_list=imp_len[hb], train_labels=np.asarray(context_dict["labels"])[hb],
            log_dir=self.log_dir, token_ckpt_dir=self.token_ckpt_dir, final_attn_ckpt_dir=self.final_attn_ckpt_dir,
            exp_name=self.exp_name, max_neg_ratio=self.max_neg_ratio, max_pos_ratio=self.max_pos_ratio,
            rng=self.rng, **self.trainer_kw)
        self.trainer.train(self.num_epochs)


class TokenEmbeddingsComponent(PipelineComponent):
    """news_embeddings from the sqlite token-state DB through the token-attention
    model (components.py:955-977): ``apply_token_attn(model_path, db_name, len(news_list))``."""

    required_keys = {"news_list", "db_name"}

    def __init__(self, model_path: Path):
        self.model_path = model_path

    def transform(self, context_dict):
        check_req_keys(self.required_keys, context_dict)
        new = context_dict.copy()
        new["news_embeddings"] = apply_token_attn(self.model_path, new["db_name"], len(new["news_list"]))
        return new


class FinalAttentionComponent(PipelineComponent):
    """Pooled cosine scores + dense ranks with FinalAttention (components.py:980-1027)."""

    required_keys = {"news_embeddings", "impression_rev_ind_array", "impression_len_list",
                     "history_rev_ind_array", "history_len_list", "history_bool"}

    def __init__(self, attention_model_path: Optional[Path] = None, dtype: Optional[torch.dtype] = None, **_):
        self.attention_model = self._load(attention_model_path)
        self.dtype = dtype

    @staticmethod
    def _load(path):
        return get_final_attention_model(path)

    def transform(self, context_dict):
        check_req_keys(self.required_keys, context_dict)
        new = context_dict.copy()
        new.update(get_final_second_attention_score(
            new["history_rev_ind_array"][0], new["history_len_list"], new["impression_rev_ind_array"][0],
            new["impression_len_list"], new["news_embeddings"], new["history_bool"], self.attention_model,
            dtype=self.dtype))
        return new


class LatentAttentionComponent(FinalAttentionComponent):
    """Same scoring with LatentAttentionModel (the pooler BASELINE's north star names)."""

    @staticmethod
    def _load(path):
        return get_latent_attention_model(path)


def labels_of(context_dict) -> np.ndarray:
    return context_dict["labels"]


# Experiments the reference's scripts import by name (scripts/eval.py:6-20,
# train_v3.py:6-17, train.py / train_v2.py) but that are outside the hot path
# (SURVEY §8(f)4): import-level placeholders only; constructing one raises.
from .out_of_scope import placeholder_class as _oos  # noqa: E402

ClassificationComponent = _oos("ClassificationComponent", "components.py:261-372", __name__, PipelineComponent)
AttentionWeightComponent = _oos("AttentionWeightComponent", "components.py:375-474", __name__, PipelineComponent)
AttentionComponent = _oos("AttentionComponent", "components.py:477-643", __name__, PipelineComponent)
AttentionReduceComponent = _oos("AttentionReduceComponent", "components.py:646-757", __name__, PipelineComponent)
NewAttentionComponent = _oos("NewAttentionComponent", "components.py:760-855", __name__, PipelineComponent)
