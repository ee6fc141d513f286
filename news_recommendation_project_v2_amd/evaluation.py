"""MIND metrics: per-impression AUC, MRR, nDCG@5, nDCG@10, averaged
(reference evaluation.py:13-98, adapted there from the official MIND evaluate.py).

Same inputs and outputs as the reference ``score``: grouped integer ranks
(``y_score = 1 / rank``) and grouped labels -> dict of mean metrics plus
``num_samples``.  Instead of a ProcessPoolExecutor running sklearn per row,
the metrics are computed for all impressions at once with segmented numpy
operations:
  AUC  = Mann-Whitney U / (P*N) with tie-averaged ranks (== sklearn's
         trapezoidal ROC AUC; nan for single-class impressions like sklearn 1.7)
  MRR  = sum(y / position) / sum(y),  nDCG@k with gains 2^y - 1, log2 discounts
Positions follow ``np.argsort(y_score)[::-1]``; impressions whose scores tie
(where numpy's unstable sort decides the order) are evaluated row by row with
exactly the reference's numpy calls so tie order matches bit for bit.
"""
from __future__ import annotations

import json
from pathlib import Path
from typing import Optional, Sequence

import numpy as np


def dcg_score(y_true, y_score, k=10):
    order = np.argsort(y_score)[::-1]
    y = np.take(y_true, order[:k])
    return np.sum((2 ** y - 1) / np.log2(np.arange(len(y)) + 2))


def ndcg_score(y_true, y_score, k=10):
    return dcg_score(y_true, y_score, k) / dcg_score(y_true, y_true, k)


def mrr_score(y_true, y_score):
    order = np.argsort(y_score)[::-1]
    y = np.take(y_true, order)
    return np.sum(y / (np.arange(len(y)) + 1)) / np.sum(y)


def _row_metrics(labels, ranks):
    """One impression, reference numerics (evaluation.py:34-54)."""
    y_true = np.asarray(labels, dtype="float32")
    y_score = np.array([1.0 / r for r in ranks], dtype=np.float64)
    if np.any(y_score < 0) or np.any(y_score > 1):
        raise ValueError("score_rslt should be int from 0 to {}".format(len(labels)))
    pos = y_true > 0
    P, N = int(pos.sum()), int((~pos).sum())
    if P == 0 or N == 0:
        auc = float("nan")
    else:
        order = np.argsort(y_score, kind="stable")
        s = y_score[order]
        r = np.empty(len(s))
        i = 0
        while i < len(s):
            j = i
            while j + 1 < len(s) and s[j + 1] == s[i]:
                j += 1
            r[i:j + 1] = (i + j) / 2.0 + 1.0
            i = j + 1
        rk = np.empty_like(r)
        rk[order] = r
        auc = (rk[pos].sum() - P * (P + 1) / 2.0) / (P * N)
    with np.errstate(invalid="ignore", divide="ignore"):
        return auc, mrr_score(y_true, y_score), ndcg_score(y_true, y_score, 5), ndcg_score(y_true, y_score, 10)


def score_row(label_sub_rank):
    """(auc, mrr, ndcg5, ndcg10) of one ``(labels, ranks, line index)`` triple
    (evaluation.py:34-54), the unit ``score`` maps over impressions."""
    labels, sub_ranks, ind = label_sub_rank
    for rank in sub_ranks:
        r = 1.0 / rank
        if r < 0 or r > 1:
            raise ValueError("Line-{}: score_rslt should be int from 0 to {}".format(ind, float(len(labels))))
    return _row_metrics(labels, sub_ranks)


def score_arrays(ranks: np.ndarray, labels: np.ndarray, offsets: np.ndarray):
    """Vectorised metrics over flat int ranks / 0-1 labels with CSR offsets.

    Returns (auc, mrr, ndcg5, ndcg10) arrays, one entry per impression.
    """
    ranks = np.asarray(ranks, dtype=np.int64)
    y = np.asarray(labels, dtype=np.float64)
    off = np.asarray(offsets, dtype=np.int64)
    n = len(off) - 1
    lens = np.diff(off)
    if np.any(ranks <= 0):
        raise ValueError("ranks must be >= 1")
    imp = np.repeat(np.arange(n), lens)
    y_score = 1.0 / ranks

    # ---- tie detection per impression (equal ranks inside one impression)
    o = np.lexsort((ranks, imp))
    rs, ims = ranks[o], imp[o]
    same = (rs[1:] == rs[:-1]) & (ims[1:] == ims[:-1])
    tie_imp = np.zeros(n, dtype=bool)
    tie_imp[ims[1:][same]] = True

    # ---- AUC by tie-averaged ascending ranks of y_score (= descending ranks)
    # ascending order of y_score within impression == descending rank value
    o2 = np.lexsort((-ranks, imp))
    r2, im2 = ranks[o2], imp[o2]
    pos_in = np.arange(len(o2)) - off[im2]
    brk = np.ones(len(o2), dtype=bool)
    brk[1:] = (r2[1:] != r2[:-1]) | (im2[1:] != im2[:-1])
    run_id = np.cumsum(brk) - 1
    run_start = pos_in[brk]
    run_len = np.bincount(run_id)
    avg = (run_start + (run_start + run_len - 1)) / 2.0 + 1.0
    asc_rank = np.empty(len(o2))
    asc_rank[o2] = avg[run_id]
    P = np.bincount(imp, weights=y, minlength=n)
    Nn = lens - P
    S = np.bincount(imp, weights=asc_rank * y, minlength=n)
    with np.errstate(invalid="ignore", divide="ignore"):
        auc = (S - P * (P + 1) / 2.0) / (P * Nn)
    auc[(P == 0) | (Nn == 0)] = np.nan

    # ---- positions in descending y_score order (valid where no ties)
    o3 = np.lexsort((ranks, imp))
    posn = np.empty(len(o3), dtype=np.int64)
    posn[o3] = np.arange(len(o3)) - off[imp[o3]]
    gains = (2.0 ** y.astype(np.float32)) - 1.0
    with np.errstate(invalid="ignore", divide="ignore"):
        mrr = np.bincount(imp, weights=y / (posn + 1), minlength=n) / P
        disc = np.log2(posn + 2.0)
        ndcg = []
        for k in (5, 10):
            dcg = np.bincount(imp, weights=np.where(posn < k, gains / disc, 0.0), minlength=n)
            # ideal DCG: labels sorted descending (tie order irrelevant)
            o4 = np.lexsort((-y, imp))
            ipos = np.arange(len(o4)) - off[imp[o4]]
            ig = gains[o4]
            idcg = np.bincount(imp[o4], weights=np.where(ipos < k, ig / np.log2(ipos + 2.0), 0.0), minlength=n)
            ndcg.append(dcg / idcg)

    # ---- rows with ties: exact reference numerics
    for i in np.nonzero(tie_imp)[0]:
        a, b = off[i], off[i + 1]
        _, m, n5, n10 = _row_metrics(y[a:b], ranks[a:b])
        mrr[i], ndcg[0][i], ndcg[1][i] = m, n5, n10
    return auc, mrr, ndcg[0], ndcg[1]


def score(preds_input: Sequence[Sequence[int]] | np.ndarray, labels_input: Sequence[Sequence[int]] | np.ndarray,
          imp_ids: Sequence[str] = (), debug_dir: Optional[Path] = None) -> dict:
    """Mean AUC / MRR / nDCG@5 / nDCG@10 over impressions (evaluation.py:57-98)."""
    lens = np.array([len(p) for p in preds_input], dtype=np.int64)
    if len(lens) != len(labels_input) or any(len(l) != n for l, n in zip(labels_input, lens)):
        raise ValueError("preds and labels must have the same grouping")
    off = np.zeros(len(lens) + 1, dtype=np.int64)
    np.cumsum(lens, out=off[1:])
    flat_r = np.concatenate([np.asarray(p, dtype=np.int64) for p in preds_input]) if len(lens) else np.zeros(0, np.int64)
    flat_y = np.concatenate([np.asarray(l, dtype=np.float64) for l in labels_input]) if len(lens) else np.zeros(0)
    aucs, mrrs, n5, n10 = score_arrays(flat_r, flat_y, off)
    if debug_dir and len(imp_ids) > 0:
        assert len(imp_ids) == len(preds_input), "Number of impression ids should be same as the number of preds"
        Path(debug_dir).mkdir(parents=True, exist_ok=True)
        with open(Path(debug_dir) / "debug_json.json", "w") as f:
            json.dump({"ImpressionID": list(imp_ids), "auc": aucs.tolist(), "mrr": mrrs.tolist(),
                       "ndcg5": n5.tolist(), "ndcg10": n10.tolist()}, f)
    return {
        "auc": np.mean(aucs).item(),
        "mrr": np.mean(mrrs).item(),
        "ndcg5": np.mean(n5).item(),
        "ndcg10": np.mean(n10).item(),
        "num_samples": len(preds_input),
    }


def score_device(ranks, labels, offsets) -> dict:
    """``score`` over flat dense ranks / 0/1 labels with CSR offsets, on the MI355X
    (nr_impression_metrics): one wave per impression instead of sklearn per row
    in a process pool (evaluation.py:57-98).  Impressions with tied ranks get
    MRR / nDCG from the host with the reference's numpy calls (their positions
    depend on np.argsort's tie order).  Accepts device or host arrays."""
    import torch

    from . import ops
    from .config import DEVICE
    dev = DEVICE
    r = torch.as_tensor(np.asarray(ranks, dtype=np.int32) if not isinstance(ranks, torch.Tensor) else ranks)
    y = torch.as_tensor(np.asarray(labels, dtype=np.float32) if not isinstance(labels, torch.Tensor) else labels)
    o = torch.as_tensor(np.asarray(offsets, dtype=np.int64) if not isinstance(offsets, torch.Tensor) else offsets)
    r, y, o = r.to(dev, torch.int32), y.to(dev, torch.float32), o.to(dev, torch.int64)
    m, tie = ops.impression_metrics(r, y, o)
    m = m.cpu().numpy()
    ties = np.nonzero(tie.cpu().numpy())[0]
    if len(ties):
        rh, yh, oh = r.cpu().numpy(), y.cpu().numpy(), o.cpu().numpy()
        with np.errstate(invalid="ignore", divide="ignore"):
            for i in ties:  # the reference's numpy calls (evaluation.py:50-53), AUC stays the device's
                a, b = oh[i], oh[i + 1]
                y_true = np.asarray(yh[a:b], dtype="float32")
                y_score = np.array([1.0 / v for v in rh[a:b]], dtype=np.float64)
                m[i, 1] = mrr_score(y_true, y_score)
                m[i, 2] = ndcg_score(y_true, y_score, 5)
                m[i, 3] = ndcg_score(y_true, y_score, 10)
    return {"auc": np.mean(m[:, 0]).item(), "mrr": np.mean(m[:, 1]).item(), "ndcg5": np.mean(m[:, 2]).item(),
            "ndcg10": np.mean(m[:, 3]).item(), "num_samples": int(len(m))}
