"""SURVEY §8(b) drop-in boundary: every Python symbol the reference's scripts and
components call (the 'Python signatures the build must keep' row) is importable
from ``news_rec_utils`` (the alias package), with the reference's parameter
names, so a reference caller switches by PYTHONPATH alone.  CPU only."""
import inspect

import pytest

import news_rec_utils  # noqa: F401  (the alias must import without a GPU)
from news_rec_utils import (components, config, data_model_helper, data_utils, evaluation, latent_attention,
                            modeling_utils, pipeline)

SURFACE = {
    data_model_helper: {
        "get_embeddings": ["model_path", "news_list", "news_text_dict"],
        "get_final_attention_eval": ["history_rev_index", "history_len_list", "news_embeddings", "model"],
        "get_cos_sim_scores": ["history_rev_index", "history_len_list", "news_rev_index", "impression_len_list",
                               "news_embeddings", "model", "query_news_embeddings"],
        "get_final_second_attention_score": ["history_rev_index", "history_len_list", "news_rev_index",
                                             "impression_len_list", "news_embeddings", "history_bool",
                                             "attention_model"],
        "apply_token_attn": ["model_path", "db_name", "num_samples"],
    },
    modeling_utils: {"get_final_attention_model": [], "get_latent_attention_model": [], "get_token_attn_model": [],
                     "get_model_and_tokenizer": [], "average_pool": [], "last_token_pool": [],
                     "FinalAttention": []},
    latent_attention: {"LatentAttentionModel": []},
    data_utils: {"load_dataset": [], "split_impressions_and_history": [], "group_items": [],
                 "rank_group_preds": [], "pad_to_maxlen": []},
    evaluation: {"score": []},
    pipeline: {"Pipeline": [], "PipelineComponent": []},
    components: {"TransformData": [], "EmbeddingsComponent": [], "SaveEmbeddingComponent": [],
                 "LoadEmbeddingComponent": [], "TokenEmbeddingsComponent": [], "FinalAttentionComponent": [],
                 "AttentionAttentionComponent": []},
}


@pytest.mark.parametrize("mod,name", [(m, n) for m, ns in SURFACE.items() for n in ns])
def test_symbol_present_with_reference_parameters(mod, name):
    obj = getattr(mod, name)
    want = SURFACE[mod][name]
    if want:
        params = list(inspect.signature(obj).parameters)
        assert params[:len(want)] == want, (name, params)


def test_config_constants():
    for k in ("EMBEDDING_DIM", "REDUCED_DIM", "DEVICE"):
        assert hasattr(config, k), k
