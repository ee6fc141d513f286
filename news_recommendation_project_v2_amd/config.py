"""Module constants and enums of the MIND hot path.

Mirrors the reference's ``src/news_rec_utils/config.py`` (constants at
config.py:24-43, enums at config.py:5-16, seeds at config.py:55-56) so that
code written against ``news_rec_utils.config`` keeps working.  Only the values
the embed -> pool -> score path reads are kept; prompts and model names are
kept verbatim because the encoder entry point (``scripts/save_emb.py``) builds
its query text from ``QUERY_INSTRUCTION``.
"""
from enum import Enum

import torch


class NewsDataset(Enum):
    """Dataset split names; values are the on-disk directory / file stems
    (reference config.py:5-10)."""

    MINDsmall_train = "MINDsmall_train"
    MINDsmall_dev = "MINDsmall_dev"
    MINDlarge_train = "MINDlarge_train"
    MINDlarge_dev = "MINDlarge_dev"
    MINDlarge_test = "MINDlarge_test"


class DataSubset(Enum):
    """Behaviour-row filter used by ``load_dataset`` (reference config.py:13-16)."""

    WITH_HISTORY = "with_history"
    WITHOUT_HISTORY = "without_history"
    ALL = "all"


# The reference picks cuda when present (config.py:19).  On PyTorch-ROCm the
# "cuda" device type is the HIP device.
DEVICE = torch.device("cuda" if torch.cuda.is_available() else "cpu")

MODEL_PATH = "intfloat/multilingual-e5-large-instruct"  # config.py:24

NEWS_TEXT_MAXLEN = 512  # config.py:27 (title tokens are truncated here)

EMBEDDING_DIM = 1024  # config.py:29

REDUCED_DIM = EMBEDDING_DIM  # config.py:31

IMPRESSION_MAXLEN = 600  # config.py:33

NUM_HIDDEN_LAYERS = 1  # config.py:35

NEWS_CLASSIFICATION_PROMPT = (
    "Please analyze the following news article to inform if the user would "
    "read the following news article.\nThe news article is: "
)

QUERY_INSTRUCTION = (
    "Instruct: Given a news article that the user has read, retrieve news "
    "articles that the user would also read \nQuery: "
)  # config.py:39

TORCH_DTYPE = torch.float32  # config.py:41

NUM_WORKERS = 4  # config.py:43

# FinalAttention hidden width (modeling_utils.py:275).
FINAL_ATTENTION_HIDDEN_DIM = 4096

# LatentAttentionModel geometry for EMBEDDING_DIM=1024 (latent_attention.py:98-104).
LATENT_NUM_LATENTS = 64
LATENT_CROSS_HEADS = 8
LATENT_CROSS_DIM_HEAD = 512
LATENT_FF_MULT = 4

SEED = 1234  # config.py:55-56

torch.manual_seed(SEED)
