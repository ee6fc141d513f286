"""Seeded MIND-shaped synthetic impressions.

No MIND data exists offline.  The generator follows the survey's recipe:
``rng = np.random.default_rng(seed)``; history length ``clip(geometric(1/33),
1, 600)``; candidates ``clip(geometric(1/37), 2, 300)``; uniform news ids
(duplicates allowed); labels ``random < 0.04`` with the first candidate forced
to 1 and the last to 0 (so every impression's AUC is defined).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np

# (n_news, n_impressions) of the public MIND splits (generator assumptions)
SHAPES = {
    "mind_small_dev": (42_416, 73_152),
    "mind_large_dev": (72_023, 376_471),
    "mind_large_test": (120_961, 2_370_727),
}


@dataclass
class Impressions:
    n_news: int
    hist_idx: np.ndarray   # int32 [H]
    hist_len: np.ndarray   # int32 [I]
    cand_idx: np.ndarray   # int32 [C]
    cand_len: np.ndarray   # int32 [I]
    labels: np.ndarray     # uint8 [C]

    @property
    def n_imp(self) -> int:
        return int(self.cand_len.shape[0])

    @property
    def n_cand(self) -> int:
        return int(self.cand_idx.shape[0])

    @property
    def n_hist(self) -> int:
        return int(self.hist_idx.shape[0])

    def hist_off(self) -> np.ndarray:
        o = np.zeros(self.n_imp + 1, dtype=np.int64)
        np.cumsum(self.hist_len, out=o[1:])
        return o

    def cand_off(self) -> np.ndarray:
        o = np.zeros(self.n_imp + 1, dtype=np.int64)
        np.cumsum(self.cand_len, out=o[1:])
        return o

    def slice(self, start: int, stop: int) -> "Impressions":
        ho, co = self.hist_off(), self.cand_off()
        return Impressions(self.n_news, self.hist_idx[ho[start]:ho[stop]], self.hist_len[start:stop],
                           self.cand_idx[co[start]:co[stop]], self.cand_len[start:stop],
                           self.labels[co[start]:co[stop]])

    def grouped_labels(self) -> list:
        co = self.cand_off()
        return [self.labels[co[i]:co[i + 1]].astype(np.int64) for i in range(self.n_imp)]


# MIND-large dev: 376,471 impressions of ~256 k users (public dataset statistics,
# an assumption here): a user's history repeats on each of the user's impressions
MIND_LARGE_DEV_USERS = 255_990


def mind_impressions(n_news: int, n_imp: int, seed: int = 1234, mean_hist: float = 33.0,
                     mean_cand: float = 37.0, max_hist: int = 600, max_cand: int = 300,
                     min_cand: int = 2, zipf: Optional[float] = None, users: Optional[int] = None) -> Impressions:
    """``users``: draw that many histories and give every impression one of
    them (each user at least once, the rest uniformly), as MIND repeats a
    user's history on all of that user's impressions; None: one independent
    history per impression (the survey's recipe, the headline workload)."""
    if users is not None:
        base = mind_impressions(n_news, n_imp, seed, mean_hist, mean_cand, max_hist, max_cand, min_cand, zipf)
        rng = np.random.default_rng(seed + 7)
        u = min(int(users), n_imp)
        pick = np.concatenate([rng.permutation(u), rng.integers(0, u, n_imp - u)]).astype(np.int64)
        ho = base.hist_off()  # user k owns impression k's history of the base draw
        hl = base.hist_len[pick]
        rows = np.repeat(ho[:-1][pick], hl) + (np.arange(int(hl.sum())) - np.repeat(np.cumsum(hl) - hl, hl))
        return Impressions(n_news, base.hist_idx[rows], hl.astype(np.int32), base.cand_idx, base.cand_len,
                           base.labels)
    rng = np.random.default_rng(seed)
    hist_len = np.clip(rng.geometric(1.0 / mean_hist, n_imp), 1, max_hist).astype(np.int32)
    cand_len = np.clip(rng.geometric(1.0 / mean_cand, n_imp), min_cand, max_cand).astype(np.int32)
    H, C = int(hist_len.sum()), int(cand_len.sum())
    if zipf is None:
        hist_idx = rng.integers(0, n_news, H, dtype=np.int32)
        cand_idx = rng.integers(0, n_news, C, dtype=np.int32)
    else:  # popularity-skewed ids for cache-sensitivity runs
        perm = rng.permutation(n_news).astype(np.int32)
        hist_idx = perm[(rng.zipf(zipf, H) - 1) % n_news]
        cand_idx = perm[(rng.zipf(zipf, C) - 1) % n_news]
    labels = (rng.random(C) < 0.04).astype(np.uint8)
    co = np.zeros(n_imp + 1, dtype=np.int64)
    np.cumsum(cand_len, out=co[1:])
    labels[co[:-1]] = 1
    labels[co[1:] - 1] = 0
    return Impressions(n_news, hist_idx, hist_len, cand_idx, cand_len, labels)


def mind_shaped(name: str = "mind_large_dev", seed: int = 1234, **kw) -> Impressions:
    n_news, n_imp = SHAPES[name]
    return mind_impressions(n_news, n_imp, seed=seed, **kw)


def to_behaviors(imps: Impressions, with_labels: bool = True, news_prefix: str = "N"):
    """Render as MIND behaviours strings (History, Impressions) for parser tests
    (token strings built once per news id, then joined per row)."""
    ho, co = imps.hist_off(), imps.cand_off()
    names = np.array([f"{news_prefix}{i}" for i in range(imps.n_news)], dtype=object)
    hist_tok = names[imps.hist_idx]
    if with_labels:
        lab = [np.array([f"{news_prefix}{i}-{y}" for i in range(imps.n_news)], dtype=object) for y in (0, 1)]
        cand_tok = np.where(imps.labels.astype(bool), lab[1][imps.cand_idx], lab[0][imps.cand_idx])
    else:
        cand_tok = names[imps.cand_idx]
    hist = [" ".join(hist_tok[ho[i]:ho[i + 1]]) if ho[i + 1] > ho[i] else None for i in range(imps.n_imp)]
    impr = [" ".join(cand_tok[co[i]:co[i + 1]]) for i in range(imps.n_imp)]
    return hist, impr


def logistic_labels(ref_scores, cand_len, seed: int = 1, slope: float = 4.0) -> np.ndarray:
    """Clicks that follow a reference score (so an AUC measures ranking quality,
    not noise around 0.5): y ~ Bernoulli(sigmoid(slope * z)), z = (s - q90(s)) /
    std(s) over all candidates (the recipe of tests/test_gpu_parity.py
    test_gpu_f32_and_bf16_vs_oracle_auc).  An impression left with one class gets
    one candidate flipped, chosen uniformly (not by score), so every impression
    has both classes and a defined AUC, as the MIND-shaped random labels do.
    Returns int64 [C]."""
    s = np.asarray(ref_scores, dtype=np.float64)
    lens = np.asarray(cand_len, dtype=np.int64)
    rng = np.random.default_rng(seed)
    z = (s - np.quantile(s, 0.9)) / (s.std() + 1e-12)
    y = (rng.random(len(s)) < 1.0 / (1.0 + np.exp(-slope * z))).astype(np.int64)
    off = np.concatenate([[0], np.cumsum(lens)])
    pos = np.add.reduceat(y, off[:-1]) if len(lens) else np.zeros(0, np.int64)
    one_class = np.nonzero((pos == 0) | (pos == lens))[0]
    pick = off[one_class] + (rng.random(len(one_class)) * lens[one_class]).astype(np.int64)
    y[pick] = 1 - y[pick]
    return y
