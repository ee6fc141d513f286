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
