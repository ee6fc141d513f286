"""On-device MIND metrics (nr_impression_metrics) against the
reference's score_row / score outputs (tests/golden/rank_score.npz, sklearn
1.7.2 roc_auc_score + the MIND mrr/ndcg functions) and the host restatement.
Tolerance 1e-12 (f64 sums in a different order; sklearn's trapezoid vs the
exact Mann-Whitney ratio)."""
import numpy as np
import pytest
import torch

from conftest import golden, unflat
from news_recommendation_project_v2_amd import evaluation

pytestmark = pytest.mark.gpu


def test_metrics_kernel_matches_reference_rows(gpu_device):
    from news_recommendation_project_v2_amd import ops
    g = golden("rank_score")
    lens = g["m_lens"]
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    r = torch.as_tensor(g["m_ranks_flat"].astype(np.int32)).to(gpu_device)
    y = torch.as_tensor(g["m_labels_flat"].astype(np.float32)).to(gpu_device)
    m, tie = ops.impression_metrics(r, y, torch.as_tensor(off).to(gpu_device))
    m, tie = m.cpu().numpy(), tie.cpu().numpy()
    want = g["m_rows"]
    for i in range(len(lens)):
        ranks = g["m_ranks_flat"][off[i]:off[i + 1]]
        assert tie[i] == int(ranks.max() < len(ranks))
        np.testing.assert_allclose(m[i, 0], want[i, 0], rtol=0, atol=1e-12, equal_nan=True)
        if not tie[i]:
            np.testing.assert_allclose(m[i, 1:], want[i, 1:], rtol=0, atol=1e-12)
    res = evaluation.score_device(g["m_ranks_flat"], g["m_labels_flat"], off)
    got = np.array([res[k] for k in ("auc", "mrr", "ndcg5", "ndcg10")])
    np.testing.assert_allclose(got, g["m_score"], rtol=0, atol=1e-12, equal_nan=True)


def test_metrics_kernel_matches_host_at_scale(gpu_device):
    rng = np.random.default_rng(5)
    n = 20000
    lens = np.clip(rng.geometric(1 / 37, n), 2, 300)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    ranks, labels = [], []
    for c in lens:
        s = rng.standard_normal(c)
        if rng.random() < 0.1:
            s[: c // 2] = np.round(s[: c // 2])  # some tied impressions
        from scipy.stats import rankdata
        ranks.append(rankdata(-s, method="dense").astype(np.int64))
        lab = (rng.random(c) < 0.05).astype(np.float64)
        lab[0] = 1
        labels.append(lab)
    r, y = np.concatenate(ranks), np.concatenate(labels)
    host = evaluation.score_arrays(r, y, off)
    dev = evaluation.score_device(r, y, off)
    want = [np.mean(h).item() for h in host]
    got = [dev[k] for k in ("auc", "mrr", "ndcg5", "ndcg10")]
    np.testing.assert_allclose(got, want, rtol=0, atol=1e-12, equal_nan=True)


def test_metrics_kernel_register_and_lds_paths(gpu_device):
    """Per-impression rows vs the host restatement across both kernel paths:
    register (<= 320 candidates, 1-5 blocks of 64) and LDS (321-2048), with
    ties, single-class rows (NaN AUC) and empty impressions."""
    from scipy.stats import rankdata
    from news_recommendation_project_v2_amd import ops
    rng = np.random.default_rng(9)
    lens = np.array([0, 1, 2, 63, 64, 65, 128, 129, 300, 320, 321, 700, 2048, 40, 40], np.int64)
    ranks, labels = [], []
    for i, c in enumerate(lens):
        s = rng.standard_normal(c)
        if i % 3 == 0:
            s = np.round(s * 2)  # ties
        ranks.append(rankdata(-s, method="dense").astype(np.int64) if c else np.zeros(0, np.int64))
        lab = (rng.random(c) < 0.1).astype(np.float64)
        if c and i != 13:
            lab[0] = 1
        if i == 14:
            lab[:] = 1  # single-class: all positive
        labels.append(lab)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    r, y = np.concatenate(ranks), np.concatenate(labels)
    m, tie = ops.impression_metrics(torch.as_tensor(r.astype(np.int32)).to(gpu_device),
                                    torch.as_tensor(y.astype(np.float32)).to(gpu_device),
                                    torch.as_tensor(off).to(gpu_device))
    m, tie = m.cpu().numpy(), tie.cpu().numpy()
    for i, c in enumerate(lens):
        if c == 0:
            assert np.isnan(m[i]).all()
            continue
        want = evaluation._row_metrics(labels[i], ranks[i])
        assert tie[i] == int(ranks[i].max() < c)
        np.testing.assert_allclose(m[i, 0], want[0], rtol=0, atol=1e-12, equal_nan=True)
        if not tie[i]:
            np.testing.assert_allclose(m[i, 1:], want[1:], rtol=0, atol=1e-12, equal_nan=True)
