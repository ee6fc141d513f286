"""CPU tests of the product's host logic (no GPU compute)."""
import re
from pathlib import Path

import numpy as np
import pytest
import torch

from conftest import REPO, golden, unflat
from news_recommendation_project_v2_amd import data_utils, evaluation, synthetic
from news_recommendation_project_v2_amd import weights as W
from news_recommendation_project_v2_amd.latent_attention import LatentAttentionModel, interleave_geglu_rows, lnfold_weights
from oracle import data_ref, pool_ref


def test_split_product_matches_reference_golden():
    g = golden("split")
    hist = [None if none else h for h, none in zip(g["history"], g["history_is_none"])]
    out = data_utils.split_impressions_and_history(list(g["impressions"]), hist)
    np.testing.assert_array_equal(out["news_list"], g["news_list"])
    for k in ("impression_rev_ind_array", "impression_len_list", "history_rev_ind_array", "history_len_list"):
        np.testing.assert_array_equal(out[k], g[k])
        assert out[k].dtype == g[k].dtype, k
    labels = [tuple(x) for x in unflat(g["labels_flat"], g["labels_len"])]
    assert [tuple(x) for x in out["labels"]] == labels
    nolab = data_utils.split_impressions_and_history(
        [" ".join(t.split("-")[0] for t in r.split()) for r in g["impressions"]], hist)
    np.testing.assert_array_equal(nolab["news_list"], g["nolab_news_list"])
    np.testing.assert_array_equal(nolab["impression_rev_ind_array"], g["nolab_impression_rev_ind_array"])
    assert nolab["labels"].size == int(g["nolab_labels_size"])


def test_split_product_matches_oracle_on_synthetic():
    imps = synthetic.mind_impressions(300, 400, seed=3)
    hist, impr = synthetic.to_behaviors(imps)
    hist[5] = None
    a = data_utils.split_impressions_and_history(impr, hist)
    b = data_ref.split_impressions_and_history(impr, hist)
    for k in a:
        if k == "labels":
            assert [tuple(x) for x in a[k]] == [tuple(x) for x in b[k]]
        else:
            np.testing.assert_array_equal(a[k], b[k])


def test_group_items_quirks():
    x = np.arange(6)
    g = data_utils.group_items(x, np.array([2, 2, 2]))
    ref = pool_ref.group(x, np.array([2, 2, 2]))
    assert g.shape == ref.shape == (3, 2)  # equal lengths -> 2-D object array, like the reference
    g2 = data_utils.group_items(x, np.array([1, 5]))
    assert g2.shape == (2,) and list(g2[1]) == [1, 2, 3, 4, 5]


def test_metrics_match_reference_golden():
    g = golden("rank_score")
    ranks = unflat(g["m_ranks_flat"], g["m_lens"])
    labels = unflat(g["m_labels_flat"], g["m_lens"])
    res = evaluation.score(ranks, labels)
    got = np.array([res[k] for k in ("auc", "mrr", "ndcg5", "ndcg10")])
    np.testing.assert_allclose(got, g["m_score"], rtol=0, atol=1e-12, equal_nan=True)
    off = data_utils.lengths_to_offsets(g["m_lens"])
    rows = np.stack(evaluation.score_arrays(g["m_ranks_flat"], g["m_labels_flat"], off), 1)
    np.testing.assert_allclose(rows, g["m_rows"], rtol=0, atol=1e-12, equal_nan=True)


def test_metrics_match_oracle_with_ties_and_long_rows():
    rng = np.random.default_rng(5)
    ranks, labels = [], []
    for i in range(300):
        c = int(rng.integers(2, 120))
        s = rng.integers(0, max(2, c // (1 + i % 4)), c)  # many ties
        ranks.append(pool_ref.dense_ranks(s.astype(np.float32), np.array([c]))[0])
        lab = (rng.random(c) < 0.1).astype(np.int64)
        lab[0], lab[-1] = 1, 0
        labels.append(lab)
    res = evaluation.score(ranks, labels)
    ref = data_ref.score(ranks, labels)
    for k in ("auc", "mrr", "ndcg5", "ndcg10"):
        assert abs(res[k] - ref[k]) < 1e-12, k


def test_weight_generator_is_deterministic():
    a = W.uniform_tensor(1234, "x", (1000,), 0.5)
    b = W.uniform_tensor(1234, "x", (1000,), 0.5)
    assert torch.equal(a, b)
    assert not torch.equal(a, W.uniform_tensor(1234, "y", (1000,), 0.5))
    assert abs(float(a.abs().max()) - 0.5) < 1e-2
    # pinned values (generator version 1)
    u = W.uniform01(1234, "pin", 3)
    assert u.shape == (3,) and np.all((u >= 0) & (u < 1))
    n = W.normal_tensor(1, "t", (20000,))
    assert abs(float(n.mean())) < 0.03 and abs(float(n.std()) - 1) < 0.03


def test_synthetic_shapes():
    imps = synthetic.mind_impressions(1000, 5000, seed=1)
    assert imps.hist_len.min() >= 1 and imps.hist_len.max() <= 600
    assert imps.cand_len.min() >= 2 and imps.cand_len.max() <= 300
    co = imps.cand_off()
    assert np.all(imps.labels[co[:-1]] == 1) and np.all(imps.labels[co[1:] - 1] == 0)
    assert abs(imps.hist_len.mean() - 33) < 3 and abs(imps.cand_len.mean() - 37.5) < 3


def test_latent_fold_equals_reference_algebra():
    """The K/V fold (A, Bt, interleaved GEGLU rows) reproduces the reference
    per-item hiddens (latent_attention.py:157-163) in float64."""
    sd = W.latent_attention_state_dict(7, ln_random=True)
    m = LatentAttentionModel()
    m.load_state_dict(sd)
    fw = m.folded_weights()
    e = W.news_table(7, 6, 1024).double()
    sd64 = {k: v.double() for k, v in sd.items()}
    want = pool_ref.latent_hiddens(sd64, e.unsqueeze(0))[0]
    y = torch.nn.functional.layer_norm(e, (1024,), fw["lnq_g"], fw["lnq_b"], 1e-5)
    s = y @ fw["A"].T
    p = torch.softmax(s.reshape(6, 8, 64), -1).reshape(6, 512)
    h1 = e + p @ fw["Bt"].T
    z = torch.nn.functional.layer_norm(h1, (1024,), fw["lnf_g"], fw["lnf_b"], 1e-5) @ fw["W1i"].T + fw["b1i"]
    z = z.reshape(6, 128, 2, 32)
    f = (z[:, :, 0] * torch.nn.functional.gelu(z[:, :, 1])).reshape(6, 4096)
    h = h1 + f @ fw["W2"].T + fw["b2"]
    np.testing.assert_allclose(h.numpy(), want.numpy(), rtol=0, atol=1e-10)


def test_lnfold_weights_reproduce_layernorm_gemm():
    """LN(a) . w_n + b_n == rstd (a . w'_n - mean u_n) + c_n  (nr_latent_transform_lnfold's
    epilogue algebra) in float64 with the bf16-rounded w' = w o gamma, to bf16
    weight-rounding accuracy; and exactly c_n for a constant row (u from the rounded w')."""
    g = torch.Generator().manual_seed(3)
    w = torch.randn(256, 1024, generator=g, dtype=torch.float64) * 0.03
    gamma = 1 + 0.2 * torch.randn(1024, generator=g, dtype=torch.float64)
    beta = 0.1 * torch.randn(1024, generator=g, dtype=torch.float64)
    b = 0.05 * torch.randn(256, generator=g, dtype=torch.float64)
    f = lnfold_weights(w, gamma, beta, b, "x")
    wf, uc = f["Wx_ln"].double(), f["ucx"].double()
    a = torch.randn(8, 1024, generator=g, dtype=torch.float64) * 2 + 0.7  # offset mean
    mean, var = a.mean(1, keepdim=True), a.var(1, unbiased=False, keepdim=True)
    rstd = 1 / torch.sqrt(var + 1e-5)
    want = torch.nn.functional.layer_norm(a, (1024,), gamma, beta, 1e-5) @ w.T + b
    got = rstd * (a @ wf.T - mean * uc[0]) + uc[1]
    # the only difference is bf16 rounding of w o gamma (relative 2^-9 per weight)
    assert (got - want).abs().max() < 2e-2 * want.abs().max()
    wexact = (w * gamma[None, :]).to(torch.bfloat16).double() / gamma[None, :]
    # exact identity: the gamma part through the rounded weights, c from the unrounded ones
    want_r = torch.nn.functional.layer_norm(a, (1024,), gamma, beta, 1e-5) @ wexact.T + b + (w - wexact) @ beta
    np.testing.assert_allclose(got.numpy(), want_r.numpy(), rtol=0, atol=1e-6)  # u, c stored f32
    np.testing.assert_allclose((0.37 * wf.sum(1) - 0.37 * uc[0]).numpy(), 0.0, atol=1e-6)
    assert f["Wx_ln"].dtype == torch.bfloat16 and f["ucx"].shape == (2, 256) and f["ucx"].dtype == torch.float32


def test_interleave_geglu_rows():
    w = torch.arange(8 * 64).reshape(128, 4)
    wi = interleave_geglu_rows(w)
    assert torch.equal(wi[:32], w[:32]) and torch.equal(wi[32:64], w[64:96])
    assert torch.equal(wi[64:96], w[32:64]) and torch.equal(wi[96:], w[96:])


def test_state_dict_keys_match_reference_layout():
    from news_recommendation_project_v2_amd.modeling_utils import FinalAttention
    fa = FinalAttention(1024, 4096)
    assert set(fa.state_dict()) == set(W.final_attention_state_dict(1))
    lm = LatentAttentionModel()
    assert list(lm.state_dict()) == list(W.latent_attention_state_dict(1))
    for k, v in W.latent_attention_state_dict(1).items():
        assert lm.state_dict()[k].shape == v.shape, k


def test_product_refuses_cpu_tensors():
    from news_recommendation_project_v2_amd._lib import NewsRecHIPError
    from news_recommendation_project_v2_amd.modeling_utils import FinalAttention
    fa = FinalAttention(1024, 4096).eval()
    with pytest.raises(NewsRecHIPError):
        fa(torch.zeros(1, 2, 1024), torch.ones(1, 2))


def test_news_rec_utils_alias():
    import news_rec_utils
    import news_rec_utils.data_model_helper as dmh
    import news_recommendation_project_v2_amd.data_model_helper as real
    assert dmh is real
    from news_rec_utils.config import EMBEDDING_DIM, NewsDataset
    assert EMBEDDING_DIM == 1024 and NewsDataset.MINDlarge_dev.value == "MINDlarge_dev"


def test_eval_collate_fn_pads_and_truncates():
    """data_utils.eval_collate_fn (reference data_utils.py:471-482) with a
    stand-in tokenizer: the texts, max_length, padding and truncation reach it."""
    from news_recommendation_project_v2_amd.data_utils import eval_collate_fn
    seen = {}

    def tok(texts, **kw):
        seen.update(kw, texts=texts)
        return "batch"

    assert eval_collate_fn(("a", "b"), tok, 7) == "batch"
    assert seen == {"texts": ["a", "b"], "max_length": 7, "padding": True, "truncation": True, "return_tensors": "pt"}


def test_distinct_segments_exact_grouping():
    """data_utils.distinct_segments (the engine's repeated-history grouping)
    against a brute-force dict of the segments: identical groups numbered by
    first occurrence, empty segments grouped together; the engine's cheap
    (length, first, last) bound never rules out a real repeat share."""
    from news_recommendation_project_v2_amd.data_utils import distinct_segments, lengths_to_offsets
    from news_recommendation_project_v2_amd.engine import DEDUPE_MIN_SHARE, _may_repeat
    from news_recommendation_project_v2_amd import synthetic
    rng = np.random.default_rng(0)
    for users, n in ((None, 800), (300, 900), (50, 400)):
        im = synthetic.mind_impressions(60, n, seed=users or 1, users=users, mean_hist=4.0)
        hl = im.hist_len.astype(np.int64).copy()
        ho = lengths_to_offsets(hl)
        keep = rng.random(n) < 0.05  # some empty histories
        hl[keep] = 0
        idx = np.concatenate([im.hist_idx[ho[i]:ho[i] + hl[i]] for i in range(n)])
        group, first = distinct_segments(idx, hl)
        off = lengths_to_offsets(hl)
        seen, bg, bf = {}, [], []
        for i in range(n):
            key = tuple(idx[off[i]:off[i + 1]])
            if key not in seen:
                seen[key] = len(seen)
                bf.append(i)
            bg.append(seen[key])
        np.testing.assert_array_equal(group, bg)
        np.testing.assert_array_equal(first, bf)
        share = 1.0 - len(first) / n
        if share >= DEDUPE_MIN_SHARE:
            assert _may_repeat(idx, hl)


def test_group_items_native_views_match_the_expression():
    """data_utils.group_items through the _nrhost extension (csrc/host/group_views.cpp)
    returns what the reference's expression np.array([items[s:e] ...], dtype=object)
    returns (data_utils.py:400-411): same shape, per-group values and dtype, views of
    `items` (a write through one shows in items), empty groups included; equal run
    lengths still give the expression's 2-D object array."""
    import numpy as np
    from news_recommendation_project_v2_amd import data_utils
    assert data_utils._nrhost() is not None, "the _nrhost extension is not built (__graft_entry__.build())"
    rng = np.random.default_rng(3)
    counts = rng.integers(0, 9, 5000)
    for dt in (np.int64, np.float32, np.int32):
        items = rng.integers(0, 100, int(counts.sum())).astype(dt)
        got = data_utils.group_items(items, counts)
        ends = np.cumsum(counts)
        want = np.array([items[s:e] for s, e in zip(ends - counts, ends)], dtype=object)
        assert got.shape == want.shape == (len(counts),) and got.dtype == object
        for g, w in zip(got, want):
            assert g.dtype == w.dtype and np.array_equal(g, w)
        got[1][:1] = 7 if len(got[1]) else 0
        if len(got[1]):
            assert items[ends[0]] == 7  # a view, as items[s:e]
    eq = data_utils.group_items(np.arange(12), np.full(4, 3))
    assert eq.shape == (4, 3)  # np.array's 2-D result for equal lengths, kept
