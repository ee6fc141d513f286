"""Data layer of the hot path: MIND behaviours -> CSR index arrays.

Mirrors the reference's ``src/news_rec_utils/data_utils.py`` functions that the
embed -> pool -> score path uses (load_dataset 26-122,
split_impressions_and_history 168-232, group_items 400-411, rank_group_preds
414-415, pad_to_maxlen 723-750, eval datasets 485-509).  Outputs are
bit-identical to the reference's, including its numpy quirks (``labels`` and
``group_items`` results built with ``np.array(..., dtype=object)``).

``to_csr`` turns the reference's (flat index, per-row length) pairs into the
device layout the HIP kernels consume: int32 row indices + int64 offsets.
"""
from __future__ import annotations

import json
from pathlib import Path
from typing import Any, Callable, Iterable, Optional, Sequence

import numpy as np
import torch
from torch.utils.data import Dataset

from .config import DataSubset, NewsDataset


def load_dataset(data_dir: Path, news_dataset: NewsDataset, num_samples: Optional[int] = None,
                 data_subset: Optional[DataSubset] = DataSubset.ALL,
                 random_state: int | np.random.Generator = 1234):
    """Read ``{data_dir}/processed/{split}/behaviors.parquet`` and ``news_text.parquet``
    (layout written by the reference's ``store_processed_data``, data_utils.py:442-455).

    Returns ``(behaviors, feature_dict)`` like data_utils.py:114-122, including
    the per-news mean entity embeddings of ``entity_embeds.pkl`` (:40-42,
    :56-99; a news with no known entity gets the 100-d zero vector).  Entity
    embeddings and category maps are optional here (they are not read by the
    embed -> pool -> score path); missing files leave those keys out.  The
    WITH_HISTORY / WITHOUT_HISTORY filter and the ``behaviors.sample`` draw
    are the reference's (:100-107), so the same ``random_state`` generator
    picks the same impressions (tests/test_dataset_golden.py).
    """
    import pandas as pd

    base = Path(data_dir) / "processed" / news_dataset.value
    behaviors = pd.read_parquet(base / "behaviors.parquet", columns=["ImpressionID", "History", "Impressions"])
    news_text = pd.read_parquet(base / "news_text.parquet").set_index("NewsID")

    def _json(p: Path) -> dict:
        return json.loads(p.read_text()) if p.is_file() else {}

    cat_dict = _json(Path(data_dir) / "categories.json")
    sub_cat_dict = _json(Path(data_dir) / "sub_categories.json")

    feats: dict[str, Any] = {"news_text_dict": news_text["news_text"].to_dict()}
    ent_path = base / "entity_embeds.pkl"
    if ent_path.is_file():
        import joblib  # the reference's own format for this file (data_utils.py:40-42)
        entity_embeds = joblib.load(ent_path)

        def mean_entity(x) -> np.ndarray:
            embeds = [] if pd.isnull(x) else [entity_embeds[e["WikidataId"]] for e in json.loads(x)
                                              if e["WikidataId"] in entity_embeds]
            return np.mean(embeds if embeds else [[0] * 100], axis=0)

        for col, key in (("Title Entities", "news_title_entity"), ("Abstract Entities", "news_abstract_entity")):
            if col in news_text:
                feats[key] = {k: mean_entity(v) for k, v in news_text[col].to_dict().items()}
    if "Title" in news_text:
        feats["news_title_dict"] = {k: "News Title: " + v for k, v in news_text["Title"].to_dict().items()}
    if "Abstract" in news_text:
        feats["news_abstract_dict"] = {k: "News Abstract: " + v
                                       for k, v in news_text["Abstract"].dropna().to_dict().items()}
    if "Category" in news_text:
        feats["news_category"] = news_text["Category"].map(cat_dict).to_dict()
    if "SubCategory" in news_text:
        feats["news_subcategory"] = news_text["SubCategory"].map(sub_cat_dict).to_dict()

    if data_subset == DataSubset.WITH_HISTORY:
        behaviors = behaviors[behaviors["History"].notna()].reset_index(drop=True)
    elif data_subset == DataSubset.WITHOUT_HISTORY:
        behaviors = behaviors[behaviors["History"].isna()].reset_index(drop=True)
    if num_samples and num_samples < len(behaviors):
        behaviors = behaviors.sample(n=num_samples, random_state=random_state, replace=False).reset_index(drop=True)
    return behaviors, feats


def split_impressions_and_history(impressions: Sequence[str], history: Sequence[Optional[str]]) -> dict[str, Any]:
    """Parse behaviours rows into first-appearance-ordered news ids and int32
    index arrays (data_utils.py:168-232).

    Per row the history ids are registered before the impression ids; a falsy
    history (None / "") contributes no history row.  Returns the reference's
    keys: news_list, impression_rev_ind_array [2, C], impression_len_list [I],
    history_rev_ind_array [2, H], history_len_list [I'], labels.
    """
    assert len(impressions) > 0, "No Impressions given"
    from .native import split_behaviors
    res = split_behaviors(impressions, history)  # C++ parser (libnewsrec_host.so)
    if res is None:
        res = split_impressions_and_history_py(impressions, history)
    if len(res["history_len_list"]) == 0:
        # the reference builds row 1 of history_rev_ind_array with np.concatenate over the
        # history rows (data_utils.py:225-227), which raises when no row has a history
        raise ValueError("need at least one array to concatenate")
    return res


def split_impressions_and_history_py(impressions: Sequence[str], history: Sequence[Optional[str]]) -> dict[str, Any]:
    """Pure-Python restatement of the same parse; used when the native parser
    declines an input (non-ASCII text, malformed labels) so that outputs and
    exceptions stay the reference's."""
    assert len(impressions) > 0, "No Impressions given"
    imps = list(impressions)
    hists = list(history)
    label_present = "-" in imps[0]
    position: dict[str, int] = {}
    news_list: list[str] = []

    def pos(nid: str) -> int:
        p = position.get(nid)
        if p is None:
            p = len(news_list)
            position[nid] = p
            news_list.append(nid)
        return p

    imp_idx: list[int] = []
    hist_idx: list[int] = []
    labels: list[tuple] = []
    hist_len: list[int] = []
    imp_len: list[int] = []
    for imp_row, hist_row in zip(imps, hists):
        if hist_row:
            toks = hist_row.split()
            hist_len.append(len(toks))
            hist_idx.extend([pos(t) for t in toks])
        toks = imp_row.split()
        if label_present:
            pairs = [t.split("-") for t in toks]
            ids = [p[0] for p in pairs]
            labels.append(tuple(int(p[1]) for p in pairs))
        else:
            ids = toks
        imp_len.append(len(ids))
        imp_idx.extend([pos(t) for t in ids])

    imp_len_a = np.array(imp_len, dtype=np.int32)
    hist_len_a = np.array(hist_len, dtype=np.int32)
    return {
        "news_list": np.array(news_list),
        "impression_rev_ind_array": np.stack([
            np.array(imp_idx, dtype=np.int32),
            np.repeat(np.arange(len(imp_len), dtype=np.int32), imp_len_a),
        ]),
        "impression_len_list": imp_len_a,
        "history_rev_ind_array": np.stack([
            np.array(hist_idx, dtype=np.int32),
            np.repeat(np.arange(len(hist_len), dtype=np.int32), hist_len_a),
        ]),
        "history_len_list": hist_len_a,
        "labels": np.array(labels, dtype=object),
    }


def _identity(x):
    return x


def group_items(items: np.ndarray, imp_counts: np.ndarray,
                func: Callable[[np.ndarray], np.ndarray] = _identity) -> np.ndarray:
    """Split ``items`` into consecutive runs of ``imp_counts`` (data_utils.py:400-411):
    ``np.array([func(items[s:e]) ...], dtype=object)``.  With the identity func, a
    1-D contiguous ``items`` and runs of differing lengths (the API's grouped ranks)
    the object array of views is built in C (_nrhost.group_views: the same views,
    dtype and base object; 59 ms -> ~10 ms at MIND-large-dev's 376 k impressions);
    equal run lengths everywhere (where np.array builds a 2-D object array), no
    runs, another func or the extension absent take the expression itself."""
    counts = np.asarray(imp_counts, dtype=np.int64)
    if func is _identity and len(counts) > 1 and isinstance(items, np.ndarray) and items.ndim == 1 \
            and items.flags.c_contiguous and int(counts.min()) != int(counts.max()):
        ext = _nrhost()
        if ext is not None:
            return ext.group_views(items, np.ascontiguousarray(counts))
    ends = np.cumsum(counts)
    starts = ends - counts
    # slice bounds as Python ints (.tolist()): iterating numpy int64 scalars costs more
    return np.array([func(items[s:e]) for s, e in zip(starts.tolist(), ends.tolist())], dtype=object)


_NRHOST = []


def _nrhost():
    """The _nrhost CPython extension (csrc/host/group_views.cpp, built by
    __graft_entry__.build()), or None when it was not built."""
    if not _NRHOST:
        try:
            from . import _nrhost as ext
        except ImportError:
            ext = None
        _NRHOST.append(ext)
    return _NRHOST[0]


def lengths_to_offsets(lengths: np.ndarray) -> np.ndarray:
    off = np.zeros(len(lengths) + 1, dtype=np.int64)
    np.cumsum(np.asarray(lengths, dtype=np.int64), out=off[1:])
    return off


_H1, _H2 = np.uint64(0x9E3779B97F4A7C15), np.uint64(0xC2B2AE3D27D4EB4F)


def distinct_segments(idx: np.ndarray, lens: np.ndarray):
    """Group identical segments of a CSR index array (same length, same ids in
    the same order): MIND repeats a user's history on every impression of that
    user.  Returns (group [n] int64, first [g] int64): segment i equals segment
    first[group[i]], groups numbered by first occurrence.  Two 64-bit
    polynomial hashes keyed with the length find candidates; every segment is
    then compared element by element with its group's first segment, so the
    grouping is exact (a hash collision falls back to no grouping)."""
    idx = np.asarray(idx, dtype=np.int64)
    lens = np.asarray(lens, dtype=np.int64)
    n = len(lens)
    if n == 0:
        return np.zeros(0, np.int64), np.zeros(0, np.int64)
    off = lengths_to_offsets(lens)
    seg = np.repeat(np.arange(n), lens)
    pos = np.arange(len(idx), dtype=np.int64) - off[:-1][seg]
    maxl = int(lens.max())
    p1, p2 = np.ones(max(maxl, 1), np.uint64), np.ones(max(maxl, 1), np.uint64)
    with np.errstate(over="ignore"):
        for k in range(1, maxl):
            p1[k] = p1[k - 1] * _H1
            p2[k] = p2[k - 1] * _H2
        v = idx.astype(np.uint64) + np.uint64(1)
        h1, h2 = np.zeros(n, np.uint64), np.zeros(n, np.uint64)
        nz = lens > 0
        if nz.any():
            h1[nz] = np.add.reduceat(v * p1[pos], off[:-1][nz])
            h2[nz] = np.add.reduceat(v * p2[pos], off[:-1][nz])
    order = np.lexsort((np.arange(n), h2, h1, lens))  # ties keep segment order: first occurrence leads
    k_l, k_1, k_2 = lens[order], h1[order], h2[order]
    new = np.ones(n, bool)
    new[1:] = (k_l[1:] != k_l[:-1]) | (k_1[1:] != k_1[:-1]) | (k_2[1:] != k_2[:-1])
    gsorted = np.cumsum(new) - 1
    first_of_g = order[new]                      # first occurrence of each group (sorted-key order)
    renum = np.empty(len(first_of_g), np.int64)  # renumber groups by first occurrence
    renum[np.argsort(first_of_g, kind="stable")] = np.arange(len(first_of_g))
    group = np.empty(n, np.int64)
    group[order] = renum[gsorted]
    first = np.sort(first_of_g)
    rep_pos = off[:-1][first[group]][seg] + pos
    if not np.array_equal(idx, idx[rep_pos]):    # a hash collision: do not group
        return np.arange(n, dtype=np.int64), np.arange(n, dtype=np.int64)
    return group, first


def rank_group_preds(pred_scores: np.ndarray, imp_counts: np.ndarray) -> np.ndarray:
    """Per-impression dense descending ranks (data_utils.py:414-415), computed by
    the HIP kernel ``nr_dense_rank`` and grouped into an object array of int64
    arrays exactly like ``group_items(..., rankdata(-x, 'dense'))``."""
    from . import ops
    from .config import DEVICE

    scores = torch.as_tensor(np.ascontiguousarray(pred_scores, dtype=np.float32)).to(DEVICE)
    # group_items slices past the end of a short score array (the reference's
    # unfiltered-lengths quirk, data_model_helper.py:442): clip like slicing does
    off = torch.as_tensor(np.minimum(lengths_to_offsets(imp_counts), len(pred_scores))).to(DEVICE)
    ranks = ops.dense_rank(scores, off).cpu().numpy().astype(np.int64)
    return group_items(ranks, imp_counts)


def pad_to_maxlen(grouped_items) -> dict[str, np.ndarray]:
    """Right-pad index groups with 0 and build the int32 mask (data_utils.py:723-750)."""
    lens = [len(g) for g in grouped_items]
    width = max(lens)
    idx = np.zeros((len(lens), width), dtype=np.int32)
    mask = np.zeros((len(lens), width), dtype=np.int32)
    for r, g in enumerate(grouped_items):
        idx[r, :lens[r]] = g
        mask[r, :lens[r]] = 1
    return {"indices": idx, "attention_mask": mask}


def expand_items(items: np.ndarray, rev_index: np.ndarray, imp_counts: np.ndarray) -> np.ndarray:
    """``items[rev_index]`` concatenated over the impression runs (data_utils.py:391-397).
    The runs tile ``rev_index`` in order, so this is one gather of its first
    ``sum(imp_counts)`` entries."""
    n = int(np.sum(imp_counts, dtype=np.int64))
    return np.asarray(items)[np.asarray(rev_index)[:n]]


def final_attention_eval_collate_fn(input, news_embeddings: torch.Tensor):
    """Padded, masked history rows of a batch of impressions (data_utils.py:784-791):
    the host-side batch the reference feeds its pooler.  The MI355X path never
    builds it (the pooling kernels read the CSR history directly);
    it is kept for callers of the reference's DataLoader pipeline."""
    padded = pad_to_maxlen(input)
    indices = torch.tensor(padded["indices"])
    attention_mask = torch.tensor(padded["attention_mask"])
    return news_embeddings[indices] * attention_mask.unsqueeze(-1), attention_mask


def to_csr(rev_index: np.ndarray, len_list: np.ndarray, device=None):
    """(flat int32 indices, per-row lengths) -> device (int32 idx, int64 offsets)."""
    idx = torch.as_tensor(np.ascontiguousarray(rev_index, dtype=np.int32))
    off = torch.as_tensor(lengths_to_offsets(len_list))
    if device is not None:
        idx, off = idx.to(device), off.to(device)
    return idx, off


def eval_collate_fn(input: Iterable[str], tokenizer, max_len: int):
    """Tokenise a batch of texts, right-padded to the batch's longest and
    truncated at max_len (data_utils.py:471-482)."""
    return tokenizer(list(input), max_length=max_len, padding=True, truncation=True, return_tensors="pt")


class AbstractTextDataset(Dataset):
    """news ids + id -> text map (data_utils.py:458-468)."""

    def __init__(self, text_list, news_text_dict: dict[str, str]):
        self.text_list = list(text_list)
        self.news_text_dict = news_text_dict

    def __len__(self):
        return len(self.text_list)

    def __getitem__(self, idx):
        raise NotImplementedError


class NewsTextDataset(AbstractTextDataset):
    """news id -> text (data_utils.py:485-487)."""

    def __getitem__(self, idx):
        return self.news_text_dict[self.text_list[idx]]


class EmbeddingDataset(Dataset):
    """Rows of an embedding table (data_utils.py:490-498)."""

    def __init__(self, embeds):
        self.embeds = embeds

    def __len__(self):
        return len(self.embeds)

    def __getitem__(self, idx):
        return self.embeds[idx]


class FinalAttentionEvalDataset(Dataset):
    """Grouped history indices per impression (data_utils.py:501-509)."""

    def __init__(self, history_rev_index: np.ndarray, history_len_list: np.ndarray):
        self.group_history = group_items(history_rev_index, history_len_list)

    def __len__(self):
        return len(self.group_history)

    def __getitem__(self, idx):
        return self.group_history[idx]


# --------------------------------------------------------------- token states
# The sqlite token-state store: table ``tensors(id INTEGER
# PRIMARY KEY, data BLOB)``, row id = news index + 1, each blob a
# ``torch.save`` of that news title's fp16 per-token hidden states
# [L_valid, 1024] (writer: modeling_utils.py:456-478 / data_model_helper.py:374-387).

def read_token_blob(blob: bytes) -> torch.Tensor:
    """One stored token-state tensor (torch.load, weights_only: executes nothing)."""
    import io
    with io.BytesIO(blob) as f:
        return torch.load(f, weights_only=True)


def tensor_pad_to_maxlen(grouped_items: Sequence[torch.Tensor]) -> dict[str, torch.Tensor]:
    """Right-pad [L_i, D] tensors to [B, L_max, D] + int32 mask (data_utils.py:753-781)."""
    lens = [len(t) for t in grouped_items]
    width = max(lens)
    emb = torch.zeros((len(lens), width) + tuple(grouped_items[0].shape[1:]), dtype=grouped_items[0].dtype)
    mask = torch.zeros((len(lens), width), dtype=torch.int32)
    for r, t in enumerate(grouped_items):
        emb[r, :lens[r]] = t
        mask[r, :lens[r]] = 1
    return {"embeddings": emb, "attention_mask": mask}


def get_embeds_from_db(conn, indices) -> dict[str, torch.Tensor]:
    """Token states of news ``indices`` (ids = index + 1), padded (data_utils.py:878-890).

    Like the reference's ``WHERE id IN (...)`` query, rows come back in
    ascending id order and missing ids are skipped."""
    ids = ",".join(str(int(i) + 1) for i in indices)
    rows = conn.execute(f"SELECT data FROM tensors WHERE id IN ({ids}) ORDER BY id;").fetchall()
    return tensor_pad_to_maxlen([read_token_blob(r[0]) for r in rows])


def iter_token_states(conn, num_items: int, chunk: int = 4096):
    """Packed token states of news 0..num_items-1 in id order: yields
    (rows [T, D] tensor, per-news lengths int64 [n]) per chunk of ids."""
    for a in range(0, num_items, chunk):
        b = min(num_items, a + chunk)
        res = conn.execute("SELECT data FROM tensors WHERE id BETWEEN ? AND ? ORDER BY id;", (a + 1, b)).fetchall()
        ts = [read_token_blob(r[0]) for r in res]
        if not ts:
            continue
        yield torch.cat(ts), np.array([len(t) for t in ts], dtype=np.int64)


class TokenAttnEvalDataset(Dataset):
    """Sequential news indices (data_utils.py:918-926)."""

    def __init__(self, num_items: int):
        self.num_items = num_items

    def __len__(self):
        return self.num_items

    def __getitem__(self, idx):
        return idx


def token_attention_eval_collate_fn(input, conn):
    """(f32 token states [B, L, D], int32 mask [B, L]) of a batch of news (data_utils.py:929-933)."""
    res = get_embeds_from_db(conn, input)
    return res["embeddings"].to(dtype=torch.float32), res["attention_mask"].to(dtype=torch.int32)


# --------------------------------------------------------------- training data (config 5)
def split_impressions_pos_neg(rng: np.random.Generator, grouped_news_rev_index, labels,
                              max_neg_ratio: Optional[float] = None, max_pos_ratio: Optional[float] = None) -> np.ndarray:
    """Balanced (positive, negative, row) triples per impression (data_utils.py:337-388).

    Per impression, with P positives and Q negatives, k = max(P, Q) (or the
    ratio-capped value): the larger side is sampled without replacement down
    to k, the smaller side is topped up to k by sampling with replacement and
    shuffled.  The generator calls (choice / permutation, same arguments, same
    order) are the reference's, so a shared ``rng`` yields identical triples.
    Returns int32 [3, sum k]: positive news, negative news, impression row.
    """
    pos_all, neg_all, counts = [], [], []
    for i, row in enumerate(labels):
        lab = np.asarray(row)
        cand = np.asarray(grouped_news_rev_index[i])
        n_pos = int(lab.sum())
        n_neg = len(lab) - n_pos
        k = max(n_pos, n_neg)
        if max_neg_ratio or max_pos_ratio:
            if max_neg_ratio and n_neg * max_neg_ratio > n_pos:
                k = int(n_pos / max_neg_ratio)
            elif max_pos_ratio and n_pos * max_pos_ratio > n_neg:
                k = int(n_neg / max_pos_ratio)
        pos = [cand[j] for j in range(len(lab)) if lab[j] != 0]
        neg = [cand[j] for j in range(len(lab)) if lab[j] == 0]
        if n_neg >= k:
            neg = rng.choice(neg, size=k, replace=False)
            pos = rng.permutation(np.append(pos, rng.choice(pos, k - n_pos)))
        else:
            pos = rng.choice(pos, size=k, replace=False)
            neg = rng.permutation(np.append(neg, rng.choice(neg, k - n_neg)))
        pos_all.extend(np.asarray(pos).tolist())
        neg_all.extend(np.asarray(neg).tolist())
        counts.append(k)
    rows = np.repeat(np.arange(len(counts)), counts).astype(np.int32)
    return np.stack([np.array(pos_all, dtype=np.int32), np.array(neg_all, dtype=np.int32), rows])


class FinalAttentionTrainDataset(Dataset):
    """(history group, positive, negative) training rows (data_utils.py:581-645).

    ``reset`` (called once per epoch) permutes impressions, draws the balanced
    pairs, and permutes whole batches except the last (ragged) one, with the
    reference's generator call order."""

    def __init__(self, history_rev_index, history_len_list, news_rev_index, impression_len_list, labels,
                 batch_size: int, max_neg_raio: Optional[float] = None, max_pos_ratio: Optional[float] = None,
                 rng=None):
        assert len(history_len_list) == len(impression_len_list), "Number of rows should match between history and news"
        assert sum(impression_len_list) == len(news_rev_index), \
            "Number of impressions should match length of impression list"
        self.group_history = group_items(history_rev_index, history_len_list)
        self.batch_size = batch_size
        self.labels = labels
        self.news_rev_index = news_rev_index
        self.impression_len_list = impression_len_list
        self.rng = rng if rng is not None else np.random.default_rng(1234)
        self.max_neg_ratio = max_neg_raio
        self.max_pos_ratio = max_pos_ratio
        self.reset()

    def __len__(self):
        return len(self.pos_neg_indices)

    def __getitem__(self, idx):
        p, n, r = self.pos_neg_indices[idx]
        return self.group_history[r], p, n

    def reset(self):
        perm = self.rng.permutation(len(self.labels))
        trip = split_impressions_pos_neg(self.rng, group_items(self.news_rev_index, self.impression_len_list)[perm],
                                         self.labels[perm], self.max_neg_ratio, self.max_pos_ratio)
        trip[2] = perm[trip[2]]
        total = trip.shape[1]
        n_batches = -(total // -self.batch_size)
        order = self.rng.permutation(n_batches - 1).tolist() + [n_batches - 1]
        sel = (np.asarray(order, dtype=np.int64)[:, None] * self.batch_size
               + np.arange(self.batch_size)[None, :]).ravel()[:total]
        self.pos_neg_indices = trip[:, sel].T

    def batches(self):
        """Row ranges of the DataLoader batches (shuffle=False, in order)."""
        n = len(self)
        return [(s, min(n, s + self.batch_size)) for s in range(0, n, self.batch_size)]


def attention_attention_train_collate_fn(input, conn):
    """Batch -> (token states, token mask, padded history indices, history mask,
    pos ‖ neg indices), all indices into the batch's sorted unique news
    (data_utils.py:893-915)."""
    from .config import NEWS_TEXT_MAXLEN
    grouped_history, pos, neg = zip(*input)
    lens = [len(h) for h in grouped_history]
    allidx = np.concatenate(list(grouped_history) + [np.asarray(pos), np.asarray(neg)])
    uniq, rev = np.unique(allidx, return_inverse=True)
    states = get_embeds_from_db(conn, uniq)
    cuts = np.cumsum(lens)
    hist_rev = np.split(rev[:cuts[-1]] if len(cuts) else rev[:0], cuts[:-1])
    padded = pad_to_maxlen(hist_rev)
    return (states["embeddings"].to(dtype=torch.float32)[:, :NEWS_TEXT_MAXLEN],
            states["attention_mask"].to(dtype=torch.int32)[:, :NEWS_TEXT_MAXLEN],
            torch.tensor(padded["indices"], dtype=torch.int32),
            torch.tensor(padded["attention_mask"], dtype=torch.int32),
            torch.tensor(rev[len(rev) - 2 * len(pos):], dtype=torch.int32))


def train_batch_csr(conn, rows, maxlen: Optional[int] = None):
    """Same batch in the device-friendly CSR form of train_step.TrainBatch:
    (last valid token row per unique news [U, D] (fp16 as stored), history
    indices int32 [Hs], offsets int64 [B+1], pos int32 [B], neg int32 [B]).
    Only the last valid token matters to the token model (attention.py:193 +
    last_token_pool), truncated at NEWS_TEXT_MAXLEN like the reference collate."""
    from .config import NEWS_TEXT_MAXLEN
    maxlen = maxlen or NEWS_TEXT_MAXLEN
    grouped_history, pos, neg = zip(*rows)
    lens = np.array([len(h) for h in grouped_history], dtype=np.int64)
    allidx = np.concatenate(list(grouped_history) + [np.asarray(pos), np.asarray(neg)])
    uniq, rev = np.unique(allidx, return_inverse=True)
    ids = ",".join(str(int(i) + 1) for i in uniq)
    res = conn.execute(f"SELECT data FROM tensors WHERE id IN ({ids}) ORDER BY id;").fetchall()
    if len(res) != len(uniq):
        # the reference fails on first_res[...] with an IndexError here; every index
        # below addresses rows of `last`, and the device gathers do not bound-check
        raise IndexError(f"token DB returned {len(res)} rows for {len(uniq)} requested news ids")
    last = torch.stack([t[min(len(t), maxlen) - 1] for t in (read_token_blob(r[0]) for r in res)])
    Hs = int(lens.sum())
    B = len(pos)
    return (last, rev[:Hs].astype(np.int32), lengths_to_offsets(lens), rev[Hs:Hs + B].astype(np.int32),
            rev[Hs + B:].astype(np.int32))


# ----------------------------------------------------------- raw TSV -> parquet
# The preprocessing step upstream of load_dataset (data_utils.py:125-165,
# 418-455, 846-875): raw MIND TSVs -> the processed parquet layout load_dataset
# reads.  Host I/O only; written for the same file names and columns.

_NEWS_COLUMNS = ["NewsID", "Category", "SubCategory", "Title", "Abstract", "URL", "Title Entities",
                 "Abstract Entities"]


def read_data(data_dir: Path, news_dataset: NewsDataset):
    """(behaviors, news, entity_embeds) from ``{data_dir}/raw/{split}/`` (data_utils.py:125-165)."""
    import pandas as pd
    raw = Path(data_dir) / "raw" / news_dataset.value
    behaviors = pd.read_csv(raw / "behaviors.tsv", sep="\t", header=None,
                            names=["ImpressionID", "UserID", "Time", "History", "Impressions"], parse_dates=["Time"])
    news = pd.read_csv(raw / "news.tsv", sep="\t", header=None, names=_NEWS_COLUMNS)
    entity = pd.read_csv(raw / "entity_embedding.vec", sep="\t", header=None)
    return behaviors, news, entity.drop(columns=[101]).set_index(0).T.to_dict("list")


def process_news(news_df):
    """Adds ``news_text = "Title: {Title}"`` (data_utils.py:430-439, config.py's passage form)."""
    news_df["news_text"] = "Title: " + news_df["Title"].astype(str)
    return news_df


def get_data(data_dir: Path, news_dataset: NewsDataset):
    """read_data + process_news (data_utils.py:418-427)."""
    behaviors, news, entity_embeds = read_data(data_dir, news_dataset)
    return behaviors, process_news(news), entity_embeds


def store_processed_data(data_dir: Path, news_dataset: NewsDataset) -> None:
    """Writes ``{data_dir}/processed/{split}/{behaviors,news_text}.parquet`` and
    ``entity_embeds.pkl`` (data_utils.py:442-455)."""
    import joblib
    behaviors, news_text, entity_embeds = get_data(data_dir, news_dataset)
    out = Path(data_dir) / "processed" / news_dataset.value
    out.mkdir(parents=True, exist_ok=True)
    behaviors.to_parquet(out / "behaviors.parquet")
    news_text.to_parquet(out / "news_text.parquet")
    joblib.dump(entity_embeds, out / "entity_embeds.pkl")


def main(argv: Optional[Sequence[str]] = None) -> None:
    """``python -m news_rec_utils.data_utils DATA_DIR SPLIT`` (data_utils.py:846-875)."""
    import argparse
    parser = argparse.ArgumentParser(description="Process news dataset and store the results.")
    parser.add_argument("data_dir", type=Path, help="Path to the directory containing data")
    parser.add_argument("news_dataset", choices=NewsDataset._member_names_, help="Select the news dataset")
    args = parser.parse_args(argv)
    if not args.data_dir.is_dir():
        parser.error(f"The path '{args.data_dir}' is not a valid directory.")
    store_processed_data(args.data_dir, NewsDataset[args.news_dataset])


# The InfoNCE / classification experiments' data helpers:
# import-level placeholders only.
from .out_of_scope import placeholder_class as _oos_cls, placeholder_function as _oos_fn  # noqa: E402

split_impressions = _oos_fn("split_impressions", "data_utils.py:235-272", __name__)
split_impressions_pos_neg_infonce = _oos_fn("split_impressions_pos_neg_infonce", "data_utils.py:275-334", __name__)
final_attention_train_infonce_collate_fn = _oos_fn("final_attention_train_infonce_collate_fn", "data_utils.py:794-817",
                                                   __name__)
final_attention_train_collate_fn = _oos_fn("final_attention_train_collate_fn", "data_utils.py:820-843", __name__)
FinalAttentionTrainInfoNCEDataset = _oos_cls("FinalAttentionTrainInfoNCEDataset", "data_utils.py:512-578", __name__,
                                             Dataset)
ClassificationTrainInfoNCEDataset = _oos_cls("ClassificationTrainInfoNCEDataset", "data_utils.py:648-685", __name__,
                                             Dataset)
ClassificationTrainDataset = _oos_cls("ClassificationTrainDataset", "data_utils.py:688-720", __name__, Dataset)
