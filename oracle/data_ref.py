"""ORACLE (test infrastructure only): reference index building and metrics.

split_impressions_and_history  data_utils.py:168-232 (pure-Python loop)
score / score_row              evaluation.py:13-98  (sklearn roc_auc_score,
                               MIND mrr / ndcg, serial instead of a process pool)
"""
from __future__ import annotations

import warnings

import numpy as np
from sklearn.metrics import roc_auc_score


def split_impressions_and_history(impressions, history) -> dict:
    assert len(impressions) > 0
    label_present = "-" in impressions[0]
    position, news_list = {}, []
    imp_rev, hist_rev, labels, hist_len, imp_len = [], [], [], [], []
    for i in range(len(impressions)):
        imp_row, hist_row = impressions[i], history[i]
        if hist_row:
            ids = hist_row.split()
            hist_len.append(len(ids))
            for nid in ids:
                if nid not in position:
                    position[nid] = len(news_list)
                    news_list.append(nid)
                hist_rev.append(position[nid])
        if label_present:
            pairs = [k.split("-") for k in imp_row.split()]
            ids = [p[0] for p in pairs]
            labels.append(tuple(int(p[1]) for p in pairs))
        else:
            ids = imp_row.split()
        imp_len.append(len(ids))
        for nid in ids:
            if nid not in position:
                position[nid] = len(news_list)
                news_list.append(nid)
            imp_rev.append(position[nid])
    return {
        "news_list": np.array(news_list),
        "impression_rev_ind_array": np.stack([np.array(imp_rev, dtype=np.int32),
                                              np.concatenate([[i] * n for i, n in enumerate(imp_len)],
                                                             dtype=np.int32)]),
        "impression_len_list": np.array(imp_len, dtype=np.int32),
        "history_rev_ind_array": np.stack([np.array(hist_rev, dtype=np.int32),
                                           np.concatenate([[i] * n for i, n in enumerate(hist_len)],
                                                          dtype=np.int32)]),
        "history_len_list": np.array(hist_len, dtype=np.int32),
        "labels": np.array(labels, dtype=object),
    }


def _dcg(y_true, y_score, k=10):
    order = np.argsort(y_score)[::-1]
    y = np.take(y_true, order[:k])
    return np.sum((2 ** y - 1) / np.log2(np.arange(len(y)) + 2))


def _mrr(y_true, y_score):
    order = np.argsort(y_score)[::-1]
    y = np.take(y_true, order)
    return np.sum(y / (np.arange(len(y)) + 1)) / np.sum(y)


def score_row(labels, ranks):
    y_true = np.array(labels, dtype="float32")
    y_score = [1.0 / r for r in ranks]
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        auc = roc_auc_score(y_true, y_score)
        with np.errstate(invalid="ignore", divide="ignore"):
            return (auc, _mrr(y_true, y_score), _dcg(y_true, y_score, 5) / _dcg(y_true, y_true, 5),
                    _dcg(y_true, y_score, 10) / _dcg(y_true, y_true, 10))


def score(preds, labels) -> dict:
    rows = [score_row(l, p) for l, p in zip(labels, preds)]
    aucs, mrrs, n5, n10 = zip(*rows)
    return {"auc": np.mean(aucs).item(), "mrr": np.mean(mrrs).item(), "ndcg5": np.mean(n5).item(),
            "ndcg10": np.mean(n10).item(), "num_samples": len(preds)}


def score_per_row(preds, labels):
    return np.array([score_row(l, p) for l, p in zip(labels, preds)], dtype=np.float64)


def impression_aucs(scores, labels, lens) -> np.ndarray:
    """Per-impression ROC AUC of score_row (evaluation.py:34-54) for every
    impression at once: score_row feeds sklearn 1/dense_rank, a strictly
    decreasing map of the score that keeps ties, so its AUC is the
    Mann-Whitney U / (P·N) of the raw scores with tie-averaged ranks (nan for a
    single-class impression, as sklearn 1.7 returns).  Pinned against score()
    in tests/test_oracle_golden.py; used where sklearn per impression would take
    minutes (376 k impressions)."""
    s = np.asarray(scores, dtype=np.float64)
    y = np.asarray(labels, dtype=np.float64)
    lens = np.asarray(lens, dtype=np.int64)
    n = len(lens)
    off = np.concatenate([[0], np.cumsum(lens)])
    imp = np.repeat(np.arange(n), lens)
    o = np.lexsort((s, imp))                        # ascending score within impression
    ss, im = s[o], imp[o]
    brk = np.ones(len(o), dtype=bool)
    brk[1:] = (ss[1:] != ss[:-1]) | (im[1:] != im[:-1])
    run = np.cumsum(brk) - 1
    pos = np.arange(len(o)) - off[im]
    start = pos[brk]
    rl = np.bincount(run)
    avg = start + (rl - 1) / 2.0 + 1.0
    r = np.empty(len(o))
    r[o] = avg[run]
    P = np.bincount(imp, weights=y, minlength=n)
    N = lens - P
    S = np.bincount(imp, weights=r * y, minlength=n)
    with np.errstate(invalid="ignore", divide="ignore"):
        auc = (S - P * (P + 1) / 2.0) / (P * N)
    auc[(P == 0) | (N == 0)] = np.nan
    return auc
