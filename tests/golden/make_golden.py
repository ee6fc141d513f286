"""Generate golden vectors by running the REAL reference (build container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [split rank final latent encoder token_attn ...]

Imports /root/reference/src/news_rec_utils with the import shims of SURVEY.md
§8(c) (transformers-5 type-hint aliases, stub dotenv/azure modules, a fixed
attention batch size because the reference's OOM probe only terminates on a
GPU), runs the reference functions of the hot path on seeded synthetic inputs
and deterministic weights (news_recommendation_project_v2_amd.weights), and
writes small .npz fixtures (inputs + outputs only, no pickles) next to this
script.  The fixtures travel; the reference never does.
"""
from __future__ import annotations

import os
import sys
import types
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
REPO = HERE.parents[1]
sys.path.insert(0, str(REPO))
REF_SRC = Path("/root/reference/src")


def import_reference():
    import transformers
    import transformers.tokenization_utils as tu
    import transformers.tokenization_utils_fast as tuf
    tuf.PreTrainedTokenizer = transformers.PreTrainedTokenizer
    tu.BatchEncoding = transformers.BatchEncoding
    dotenv = types.ModuleType("dotenv")
    dotenv.load_dotenv = lambda *a, **k: None
    sys.modules["dotenv"] = dotenv
    az, st, bl = (types.ModuleType(n) for n in ("azure", "azure.storage", "azure.storage.blob"))

    class _NoAzure:
        def __init__(self, *a, **k):
            raise RuntimeError("azure is not available offline")

    bl.ContainerClient = bl.BlobClient = _NoAzure
    sys.modules.update({"azure": az, "azure.storage": st, "azure.storage.blob": bl})
    sys.path.insert(0, str(REF_SRC))
    import news_rec_utils.data_model_helper as dmh
    import news_rec_utils.data_utils as du
    import news_rec_utils.evaluation as ev
    import news_rec_utils.latent_attention as la
    import news_rec_utils.modeling_utils as mu
    dmh.get_attention_inference_batch_size = lambda model: 256  # -> 128 per batch (// 2)
    return dmh, du, ev, la, mu


def flat(obj_arr):
    lens = np.array([len(x) for x in obj_arr], dtype=np.int64)
    vals = np.concatenate([np.asarray(x) for x in obj_arr]) if len(lens) else np.zeros(0)
    return vals, lens


def gen_split(du):
    rng = np.random.default_rng(7)
    hist, imps = [], []
    for i in range(60):
        hn = int(rng.integers(0, 6))
        hist.append(None if (hn == 0 or i % 13 == 5) else " ".join(f"N{int(x)}" for x in rng.integers(0, 40, hn)))
        cn = 1 if i % 11 == 3 else int(rng.integers(2, 8))
        imps.append(" ".join(f"N{int(x)}-{int(rng.random() < 0.3)}" for x in rng.integers(0, 40, cn)))
    hist[0] = "N1 N2 N1"  # repeated id inside one history
    out = du.split_impressions_and_history(imps, hist)
    labels_flat, labels_len = flat(out["labels"]) if out["labels"].dtype == object and out["labels"].ndim == 1 \
        else (np.concatenate(list(out["labels"])), np.array([len(x) for x in out["labels"]]))
    nolab = du.split_impressions_and_history([" ".join(t.split("-")[0] for t in r.split()) for r in imps], hist)
    np.savez_compressed(
        HERE / "split.npz",
        history=np.array(["" if h is None else h for h in hist]), history_is_none=np.array([h is None for h in hist]),
        impressions=np.array(imps),
        news_list=out["news_list"], impression_rev_ind_array=out["impression_rev_ind_array"],
        impression_len_list=out["impression_len_list"], history_rev_ind_array=out["history_rev_ind_array"],
        history_len_list=out["history_len_list"], labels_flat=labels_flat.astype(np.int64), labels_len=labels_len,
        nolab_news_list=nolab["news_list"], nolab_impression_rev_ind_array=nolab["impression_rev_ind_array"],
        nolab_labels_size=np.array(nolab["labels"].size))


def gen_rank_and_score(du, ev):
    rng = np.random.default_rng(11)
    counts = np.array([1, 2, 5, 7, 3, 64, 65, 130, 4, 9], dtype=np.int32)
    scores = rng.standard_normal(int(counts.sum())).astype(np.float32)
    scores[3] = scores[4]           # ties inside impressions
    scores[10:14] = scores[9]
    scores[100:120] = 0.25
    scores[200] = -0.0
    scores[201] = 0.0
    grouped = du.rank_group_preds(scores, counts)
    ranks_flat, ranks_len = flat(grouped)
    # metrics on MIND-like rows with labels, incl. a single-class row (-> nan AUC)
    lab_rows, rank_rows = [], []
    for i in range(40):
        c = int(rng.integers(2, 30))
        lab = (rng.random(c) < 0.2).astype(int)
        lab[0] = 1
        if i != 7:
            lab[-1] = 0
        else:
            lab[:] = 1
        s = rng.standard_normal(c).astype(np.float32)
        if i % 5 == 0:
            s[1] = s[0]
        lab_rows.append(tuple(int(x) for x in lab))
        rank_rows.append(du.rankdata(-s, method="dense"))
    res = ev.score(rank_rows, lab_rows)
    res_ok = ev.score([r for i, r in enumerate(rank_rows) if i != 7], [l for i, l in enumerate(lab_rows) if i != 7])
    rows = np.array([ev.score_row((l, r, i)) for i, (l, r) in enumerate(zip(lab_rows, rank_rows))])
    rf, rl = flat(rank_rows)
    lf, ll = flat(lab_rows)
    np.savez_compressed(HERE / "rank_score.npz", scores=scores, counts=counts, ranks_flat=ranks_flat.astype(np.int64),
                        ranks_len=ranks_len, m_ranks_flat=rf.astype(np.int64), m_lens=rl, m_labels_flat=lf.astype(np.int64),
                        m_rows=rows, m_score=np.array([res[k] for k in ("auc", "mrr", "ndcg5", "ndcg10")]),
                        m_score_ok=np.array([res_ok[k] for k in ("auc", "mrr", "ndcg5", "ndcg10")]))


def gen_pooler(dmh, model, sd_seed_name, pooler, n_news=512, n_imp=64, extra_unpooled=False):
    from news_recommendation_project_v2_amd import weights as W
    rng = np.random.default_rng(1234 if pooler == "final" else 4321)
    h = np.clip(rng.geometric(1 / 20.0, n_imp), 1, 600).astype(np.int32)
    c = np.clip(rng.geometric(1 / 37.0, n_imp), 2, 300).astype(np.int32)
    h[5] = 1
    h[6] = max(int(h[6]), 200)
    hi = rng.integers(0, n_news, int(h.sum())).astype(np.int32)
    ci = rng.integers(0, n_news, int(c.sum())).astype(np.int32)
    table = W.news_table(1234, n_news, 1024, name=f"golden_news_{pooler}")
    with torch.no_grad():
        scores = dmh.get_cos_sim_scores(hi, h, ci, c, table, model).numpy()
        # two-table path (data_model_helper.py:189-196): history pooled from the query table
        qtable = W.news_table(4321, n_news, 1024, name=f"golden_query_{pooler}")
        scores_2tab = dmh.get_cos_sim_scores(hi, h, ci, c, table, model, query_news_embeddings=qtable).numpy()
        users = dmh.get_final_attention_eval(hi, h, table, model).numpy()
        fs = dmh.get_final_second_attention_score(hi, h, ci, c, table, __import__("pandas").Series(np.ones(n_imp, bool)),
                                                  model)
    rf, rl = flat(fs["grouped_scores"])
    extra = {}
    if extra_unpooled:
        with torch.no_grad():
            e = table[torch.tensor(np.arange(8).reshape(2, 4))]
            extra["unpooled_in_rows"] = np.arange(8).reshape(2, 4)
            extra["unpooled_out"] = model(e, None).numpy()
    np.savez_compressed(HERE / f"pool_{pooler}.npz", n_news=n_news, table_name=f"golden_news_{pooler}",
                        weight_seed=1234, hist_idx=hi, hist_len=h, cand_idx=ci, cand_len=c, scores=scores, users=users,
                        fs_scores=fs["scores"], fs_ranks_flat=rf.astype(np.int64), fs_ranks_len=rl,
                        query_table_seed=4321, query_table_name=f"golden_query_{pooler}", scores_2tab=scores_2tab,
                        **extra)


ENC_LENS = [2, 7, 20, 31, 32, 33, 45, 64, 65, 130]


def encoder_inputs(vocab: int, seed: int = 99):
    rng = np.random.default_rng(seed)
    seqs = []
    for L in ENC_LENS:
        mid = rng.integers(5, vocab, L - 2) if L > 2 else np.zeros(0, np.int64)
        seqs.append(np.concatenate([[0], mid, [2]]).astype(np.int64))
    return seqs


def gen_encoder(mu, n_layers: int, vocab: int = 1000, fp16_weights: bool = False):
    """transformers 5.15 XLMRobertaModel (third-party, e5-large-instruct's
    architecture) with deterministic weights, run through the reference's
    get_text_embed_eval (modeling_utils.py:282-300: average_pool; saved as
    emb_mean) + F.normalize (data_model_helper.py:65-78; saved as emb).
    fp16_weights: every parameter rounded to fp16 and computed in f32 — the
    reference's GPU numerics (fp16 weights, modeling_utils.py:98, under an f32
    autocast, :285-290)."""
    import torch.nn.functional as F
    from transformers import BatchEncoding, XLMRobertaConfig, XLMRobertaModel
    from news_recommendation_project_v2_amd import weights as W
    cfg = XLMRobertaConfig(vocab_size=vocab, hidden_size=1024, num_hidden_layers=n_layers, num_attention_heads=16,
                           intermediate_size=4096, max_position_embeddings=514, layer_norm_eps=1e-5,
                           type_vocab_size=1, pad_token_id=1, hidden_act="gelu")
    cfg.architectures = ["XLMRobertaModel"]
    model = XLMRobertaModel(cfg, add_pooling_layer=False)
    sd = W.xlmr_state_dict(1234, n_layers, vocab)
    if fp16_weights:
        sd = {k: v.half().float() for k, v in sd.items()}
    missing, unexpected = model.load_state_dict(sd, strict=False)
    assert not unexpected and all("position_ids" in k or "token_type_ids" in k for k in missing), (missing, unexpected)
    model.eval()
    seqs = encoder_inputs(vocab)
    width = max(len(s) for s in seqs)
    ids = torch.ones((len(seqs), width), dtype=torch.long)
    mask = torch.zeros((len(seqs), width), dtype=torch.long)
    for i, s in enumerate(seqs):
        ids[i, :len(s)] = torch.tensor(s)
        mask[i, :len(s)] = 1
    batches = [BatchEncoding({"input_ids": ids[:5], "attention_mask": mask[:5]}),
               BatchEncoding({"input_ids": ids[5:], "attention_mask": mask[5:]})]
    with torch.no_grad():
        mean = mu.get_text_embed_eval(model, batches)
        emb = F.normalize(mean, p=2, dim=1).numpy()
    name = f"encoder_l{n_layers}" + ("_f16w" if fp16_weights else "")
    np.savez_compressed(HERE / f"{name}.npz", n_layers=n_layers, vocab=vocab, weight_seed=1234,
                        fp16_weights=fp16_weights, ids=np.concatenate(seqs).astype(np.int32),
                        lens=np.array(ENC_LENS, np.int64), emb=emb, emb_mean=mean.numpy())


TOKEN_CASES = {"ragged": [1, 5, 9, 12], "full": [8, 8, 8], "empty_row": [0, 3, 6]}


def gen_token_attn(dmh, du, mu):
    """FirstAttentionPoolFunc(last_token_pool) (modeling_utils.py:498-524) on
    fp16-valued token states (the sqlite blobs are fp16), for ragged, all-full
    (left-padding branch of last_token_pool) and an all-zero mask row; plus the
    reference's own apply_token_attn over a sqlite token DB written in the
    reference layout (id = index + 1, torch.save'd fp16 [L, 1024] blobs)."""
    import io
    import sqlite3
    import tempfile
    from news_recommendation_project_v2_amd import weights as W
    model = mu.FirstAttentionPoolFunc(pool_func=mu.last_token_pool, embedding_dim=1024, num_layers=1)
    model.load_state_dict(W.token_attn_state_dict(1234))
    model.eval()
    out = {}
    for name, lens in TOKEN_CASES.items():
        width = max(lens)
        x = (W.normal_tensor(77, f"tok_{name}", (len(lens), width, 1024)) * 3.0 + 0.5).half()
        m = torch.zeros((len(lens), width), dtype=torch.int32)
        for i, n in enumerate(lens):
            m[i, :n] = 1
            x[i, n:] = 0
        with torch.no_grad():
            y = model(x.float(), m).numpy()
        out[f"{name}_x"], out[f"{name}_mask"], out[f"{name}_out"] = x.numpy(), m.numpy(), y
    # sqlite path through the reference's apply_token_attn
    lens = [3, 1, 7, 2, 5, 4, 6]
    dmh.get_token_attention_inference_batch_size = lambda model: 13  # -> batch 3 (the OOM probe is GPU-only)
    states = [(W.normal_tensor(78, f"db_{i}", (n, 1024)) * 2.0).half() for i, n in enumerate(lens)]
    sd_path = Path(tempfile.mkdtemp()) / "token_attn.pt"
    torch.save(model.state_dict(), sd_path)
    db = sd_path.with_name("tokens.db")
    with sqlite3.connect(db) as conn:
        conn.execute("CREATE TABLE tensors (id INTEGER PRIMARY KEY, data BLOB)")
        for t in states:
            buf = io.BytesIO()
            torch.save(t, buf)
            conn.execute("INSERT INTO tensors (data) VALUES (?)", (buf.getvalue(),))
    with torch.no_grad():
        db_out = dmh.apply_token_attn(sd_path, db, len(lens)).numpy()
    np.savez_compressed(HERE / "token_attn.npz", weight_seed=1234, db_lens=np.array(lens, np.int64),
                        db_states=torch.cat(states).numpy(), db_out=db_out, **out)


TRAIN_SAMPLE = 2048  # sampled elements per parameter tensor kept in the fixture


def train_fixture_data(n_news=40, n_imp=24, seed=21):
    """Tiny MIND-shaped training set: token-state lengths, histories, candidates
    with >= 1 positive and >= 1 negative per impression."""
    rng = np.random.default_rng(seed)
    tok_lens = rng.integers(1, 13, n_news)
    h = rng.integers(1, 9, n_imp)
    c = rng.integers(3, 9, n_imp)
    hist = rng.integers(0, n_news, int(h.sum())).astype(np.int32)
    cand = rng.integers(0, n_news, int(c.sum())).astype(np.int32)
    labels = []
    for ci in c:
        lab = (rng.random(ci) < 0.3).astype(int)
        lab[0], lab[-1] = 1, 0
        labels.append(tuple(int(x) for x in lab))
    return tok_lens, h.astype(np.int32), c.astype(np.int32), hist, cand, labels


def sample_idx(numel: int, name: str) -> np.ndarray:
    return np.random.default_rng(5).integers(0, numel, TRAIN_SAMPLE)


def gen_train(dmh, du, mu):
    """Config 5 (scripts/train_v3.py): the reference's FinalAttentionTrainDataset
    batching, its collate fn, one hand-run step of the train_one_epoch body
    (trainer.py:1044-1069) with the reference modules, and a full
    AttentionAttentionTrainer.train_one_epoch, all with dropout p = 0 (the
    reference's nn.Dropout stream cannot be reproduced; the HIP path's own
    dropout is checked against oracle/train_ref.py instead)."""
    import io
    import os
    import sqlite3
    import tempfile
    import torch.nn.functional as F
    import news_rec_utils.trainer as tr
    from news_recommendation_project_v2_amd import weights as W
    tok_lens, h, c, hist, cand, labels = train_fixture_data()
    states = [(W.normal_tensor(91, f"train_tok_{i}", (int(n), 1024)) * 2.0 + 0.3).half() for i, n in enumerate(tok_lens)]
    tmp = Path(tempfile.mkdtemp())
    db = tmp / "train_tokens.db"
    with sqlite3.connect(db) as conn:
        conn.execute("CREATE TABLE tensors (id INTEGER PRIMARY KEY, data BLOB)")
        for t in states:
            buf = io.BytesIO()
            torch.save(t, buf)
            conn.execute("INSERT INTO tensors (data) VALUES (?)", (buf.getvalue(),))
    lab_arr = np.empty(len(labels), dtype=object)
    lab_arr[:] = labels
    BS = 8

    def models():
        tm = mu.FirstAttentionPoolFunc(pool_func=mu.last_token_pool, embedding_dim=1024, num_layers=1)
        tm.load_state_dict(W.token_attn_state_dict(1234))
        fa = mu.FinalAttention(reduced_dim=1024, hidden_dim=4096)
        fa.load_state_dict(W.final_attention_state_dict(1234))
        for m in (tm, fa):
            for mod in m.modules():
                if isinstance(mod, torch.nn.Dropout):
                    mod.p = 0.0
        return tm, fa

    # (a) batching + (b) collate of batch 0
    ds = du.FinalAttentionTrainDataset(hist, h, cand, c, lab_arr, batch_size=BS, rng=np.random.default_rng(1234))
    pni = ds.pos_neg_indices.copy()
    rows0 = [ds[i] for i in range(min(BS, len(ds)))]
    with sqlite3.connect(db) as conn:
        tok, tmask, hidx, hmask, pn = du.attention_attention_train_collate_fn(rows0, conn=conn)
    # (c) one step of the loop body with the reference modules
    tm, fa = models()
    tm.train(); fa.train()
    opt = torch.optim.AdamW(list(tm.parameters()) + list(fa.parameters()), lr=1e-6)
    first_res = tm(tok.float(), tmask)
    second_res = first_res[hidx] * hmask.unsqueeze(-1)
    outputs = fa(second_res, hmask)
    res = F.cosine_similarity(outputs.repeat((2, 1)), first_res[pn])
    loss = torch.nn.MarginRankingLoss(2)(*torch.chunk(res, 2), torch.tensor([1], dtype=torch.float32))
    loss.backward()
    named = {("ln." + k.split(".")[-1] if k.startswith("encoder.layer.0.g_mlp_layernorm") else k): p
             for k, p in list(tm.named_parameters()) + list(fa.named_parameters()) if p.grad is not None}
    grads = {k: p.grad.detach().clone() for k, p in named.items()}
    total = torch.nn.utils.clip_grad_norm_(list(tm.parameters()) + list(fa.parameters()), max_norm=0.5)
    opt.step()
    out = {"step_loss": np.array(float(loss)), "step_total_norm": np.array(float(total)),
           "pos_neg_indices": pni, "tok_lens": tok_lens, "hist": hist, "hist_len": h, "cand": cand, "cand_len": c,
           "labels_flat": np.concatenate([np.array(l) for l in labels]), "batch_size": np.array(BS),
           "b0_hidx": hidx.numpy(), "b0_hmask": hmask.numpy(), "b0_pn": pn.numpy(), "b0_tmask": tmask.numpy(),
           "step_grad_names": np.array(sorted(grads))}
    for k in sorted(grads):
        g = grads[k].reshape(-1).numpy()
        si = sample_idx(g.size, k)
        out[f"grad_sum:{k}"] = np.array(float(grads[k].double().sum()))
        out[f"grad_sq:{k}"] = np.array(float((grads[k].double() ** 2).sum()))
        out[f"grad_idx:{k}"] = si
        out[f"grad_val:{k}"] = g[si]
        pa = named[k].detach().reshape(-1).numpy()
        out[f"step_param_val:{k}"] = pa[si]
    # (d) the reference trainer for one epoch (Azure client stubbed; OOM-probed batch size fixed)
    os.environ.update({"ACCOUNT_URL": "stub", "CONTAINER_NAME": "stub", "BLOB_SAS_TOKEN": "stub"})

    class _Container:
        def __init__(self, *a, **k):
            pass

        def upload_blob(self, *a, **k):
            pass

    tr.ContainerClient = _Container
    tr.get_attention_attention_train_batch_size = lambda **k: BS
    tm, fa = models()
    trainer = tr.AttentionAttentionTrainer(str(db), tm, fa, hist, h, cand, c, lab_arr, rng=np.random.default_rng(1234))
    assert np.array_equal(trainer.train_dataset.pos_neg_indices, pni)
    ep_loss = trainer.train_one_epoch()
    out["epoch_loss"] = np.array(float(ep_loss))
    for k, p in list(tm.named_parameters()) + list(fa.named_parameters()):
        key = "ln." + k.split(".")[-1] if k.startswith("encoder.layer.0.g_mlp_layernorm") else k
        if key not in grads:
            continue
        pa = p.detach().reshape(-1).numpy()
        out[f"epoch_param_val:{key}"] = pa[sample_idx(pa.size, key)]
    trainer.connection.close()
    np.savez_compressed(HERE / "train_step.npz", weight_seed=1234, **out)


def dataset_inputs(seed: int = 31, n_news: int = 60, n_rows: int = 240):
    """A tiny processed MIND split in the reference's on-disk layout
    (store_processed_data, data_utils.py:442-455): behaviours rows (some with
    no history), news text / title / abstract (some missing) / category /
    subcategory / entity JSON columns, the WikidataId -> 100-d entity table
    (some ids unknown), and the category maps."""
    rng = np.random.default_rng(seed)
    news = [f"N{i}" for i in range(1, n_news + 1)]
    cats, subs = ["news", "sports", "finance", "travel", "video"], [f"sub{i}" for i in range(7)]
    qids = [f"Q{i}" for i in range(40)]
    known = qids[:30]

    def ents():
        if rng.random() < 0.25:
            return None
        return "[" + ", ".join('{"Label": "x", "WikidataId": "%s"}' % q for q in rng.choice(qids, int(rng.integers(1, 4)))) + "]"

    news_cols = {
        "NewsID": news,
        "Category": [cats[int(i)] for i in rng.integers(0, len(cats), n_news)],
        "SubCategory": [subs[int(i)] for i in rng.integers(0, len(subs), n_news)],
        "Title": [f"title {i} " + "w" * int(rng.integers(1, 9)) for i in range(n_news)],
        "Abstract": [None if rng.random() < 0.2 else f"abstract {i}" for i in range(n_news)],
        "Title Entities": [ents() for _ in range(n_news)],
        "Abstract Entities": [ents() for _ in range(n_news)],
    }
    news_cols["news_text"] = [f"Title: {t}" for t in news_cols["Title"]]
    hist, imps = [], []
    for i in range(n_rows):
        h = rng.choice(news, int(rng.integers(1, 9)))
        hist.append(None if rng.random() < 0.3 else " ".join(h))
        c = rng.choice(news, int(rng.integers(2, 9)))
        lab = (rng.random(len(c)) < 0.3).astype(int)
        imps.append(" ".join(f"{n}-{int(y)}" for n, y in zip(c, lab)))
    entity = {q: rng.standard_normal(100).tolist() for q in known}
    return news_cols, {"ImpressionID": np.arange(1, n_rows + 1), "History": hist, "Impressions": imps}, entity, \
        {c: i for i, c in enumerate(cats)}, {s: i for i, s in enumerate(subs)}


def write_dataset(root: Path, split: str, news_cols, beh_cols, entity, cat_map, sub_map) -> None:
    import joblib
    import pandas as pd
    d = root / "processed" / split
    d.mkdir(parents=True, exist_ok=True)
    pd.DataFrame(news_cols).to_parquet(d / "news_text.parquet")
    pd.DataFrame(beh_cols).to_parquet(d / "behaviors.parquet")
    joblib.dump(entity, d / "entity_embeds.pkl")
    (root / "categories.json").write_text(__import__("json").dumps(cat_map))
    (root / "sub_categories.json").write_text(__import__("json").dumps(sub_map))


DATASET_CASES = [  # (split, num_samples, subset) run in this order on ONE rng, as scripts/eval.py:38-52 does
    ("MINDsmall_train", 50, "WITH_HISTORY"),
    ("MINDsmall_dev", 40, "WITH_HISTORY"),
    ("MINDsmall_dev", None, "ALL"),
    ("MINDsmall_dev", 30, "WITHOUT_HISTORY"),
]


def gen_dataset(du):
    """Config 1 (scripts/eval.py:38-52): the reference's load_dataset on a tiny
    processed split (WITH_HISTORY / ALL / WITHOUT_HISTORY, behaviors.sample
    with a shared np.random.Generator) followed by its TransformData
    (components.py:45-114); inputs and every output array are stored."""
    import tempfile
    import news_rec_utils.components as comp
    import news_rec_utils.config as rc
    news_cols, beh_cols, entity, cat_map, sub_map = dataset_inputs()
    root = Path(tempfile.mkdtemp())
    for split in {c[0] for c in DATASET_CASES}:
        write_dataset(root, split, news_cols, beh_cols, entity, cat_map, sub_map)
    rng = np.random.default_rng(1234)
    out = {}
    for k, (split, n, subset) in enumerate(DATASET_CASES):
        beh, feats = du.load_dataset(root, rc.NewsDataset[split], num_samples=n, data_subset=rc.DataSubset[subset],
                                     random_state=rng)
        out[f"c{k}_ImpressionID"] = beh["ImpressionID"].to_numpy()
        try:
            ctx = comp.TransformData().transform({"behaviors": beh, **feats})
        except ValueError as e:  # no history row at all: the reference's np.concatenate([]) raises
            out[f"c{k}_error"] = np.array(f"ValueError: {e}")
            continue
        lab_flat, lab_len = flat(ctx["labels"])
        out.update({f"c{k}_news_list": np.asarray(ctx["news_list"]),
                    f"c{k}_impression_rev_ind_array": ctx["impression_rev_ind_array"],
                    f"c{k}_impression_len_list": ctx["impression_len_list"],
                    f"c{k}_history_rev_ind_array": ctx["history_rev_ind_array"],
                    f"c{k}_history_len_list": ctx["history_len_list"],
                    f"c{k}_labels_flat": lab_flat.astype(np.int64), f"c{k}_labels_len": lab_len,
                    f"c{k}_history_bool": ctx["history_bool"].to_numpy(),
                    f"c{k}_title_entity_embed": ctx["title_entity_embed"].numpy(),
                    f"c{k}_abstract_entity_embed": ctx["abstract_entity_embed"].numpy(),
                    f"c{k}_cat_indices": ctx["cat_indices"].numpy(), f"c{k}_subcat_indices": ctx["subcat_indices"].numpy()})
        keys = sorted(feats["news_title_dict"])[:5]
        out[f"c{k}_title_keys"] = np.array(keys)
        out[f"c{k}_title_vals"] = np.array([feats["news_title_dict"][x] for x in keys])
        akeys = sorted(feats["news_abstract_dict"])
        out[f"c{k}_abstract_keys"] = np.array(akeys)
    ent_ids = sorted(entity)
    np.savez_compressed(
        HERE / "dataset.npz", cases=np.array([f"{s}|{n}|{b}" for s, n, b in DATASET_CASES]),
        news_cols=np.array(list(news_cols)),
        **{f"news_{c}": np.array(["<NONE>" if v is None else v for v in news_cols[c]]) for c in news_cols},
        beh_ImpressionID=beh_cols["ImpressionID"],
        beh_History=np.array(["<NONE>" if v is None else v for v in beh_cols["History"]]),
        beh_Impressions=np.array(beh_cols["Impressions"]),
        entity_ids=np.array(ent_ids), entity_vecs=np.array([entity[q] for q in ent_ids]),
        cat_keys=np.array(list(cat_map)), sub_keys=np.array(list(sub_map)), **out)


def gen_imports():
    """The reference's Python API surface, read with ``ast`` (no import of the reference):
    ``scripts``: the exact ``from news_rec_utils... import ...`` lists of its entry
    scripts (scripts/*.py) as [module, name, line]; ``package``: every top-level
    class / def / assigned name of each src/news_rec_utils module.
    tests/test_api_surface.py resolves every name against the alias package."""
    import ast
    import json
    scripts, package = {}, {}
    for script in sorted((REF_SRC.parent / "scripts").glob("*.py")):
        names = []
        for node in ast.walk(ast.parse(script.read_text())):
            if isinstance(node, ast.ImportFrom) and (node.module or "").split(".")[0] == "news_rec_utils":
                names += [[node.module, a.name, node.lineno] for a in node.names]
            elif isinstance(node, ast.Import):
                names += [[a.name, None, node.lineno] for a in node.names if a.name.split(".")[0] == "news_rec_utils"]
        scripts[f"scripts/{script.name}"] = names
    for mod in sorted((REF_SRC / "news_rec_utils").glob("*.py")):
        names = []
        for node in ast.parse(mod.read_text()).body:
            if isinstance(node, (ast.FunctionDef, ast.ClassDef)):
                names.append([node.name, node.lineno])
            elif isinstance(node, ast.Assign):
                names += [[t.id, node.lineno] for t in node.targets if isinstance(t, ast.Name)]
        package[mod.stem] = names
    lines = ["{", ' "scripts": {']
    lines.append(",\n".join(f"  {json.dumps(k)}: {json.dumps(v)}" for k, v in scripts.items()))
    lines += [" },", ' "package": {']
    lines.append(",\n".join(f"  {json.dumps(k)}: {json.dumps(v)}" for k, v in package.items()))
    lines += [" }", "}"]
    text = "\n".join(lines) + "\n"
    json.loads(text)
    (HERE / "api_surface.json").write_text(text)


GENERATORS = ("split", "rank", "final", "latent", "encoder", "token_attn", "train", "dataset", "imports")


def main():
    assert REF_SRC.is_dir(), "the reference is only available in the build container"
    os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
    torch.set_num_threads(8)
    which = set(sys.argv[1:]) or set(GENERATORS)
    if "imports" in which:
        gen_imports()
        if which == {"imports"}:
            return
    dmh, du, ev, la, mu = import_reference()
    from news_recommendation_project_v2_amd import weights as W
    if "split" in which:
        gen_split(du)
    if "rank" in which:
        gen_rank_and_score(du, ev)
    if "final" in which:
        fa = mu.FinalAttention(reduced_dim=1024, hidden_dim=4096)
        fa.load_state_dict(W.final_attention_state_dict(1234))
        fa.eval()
        gen_pooler(dmh, fa, "final", "final")
    if "latent" in which:
        lm = la.LatentAttentionModel()
        lm.load_state_dict(W.latent_attention_state_dict(1234, ln_random=True))
        lm.eval()
        gen_pooler(dmh, lm, "latent", "latent", extra_unpooled=True)
    if "encoder" in which:
        gen_encoder(mu, 2)
        gen_encoder(mu, 24)
        gen_encoder(mu, 24, fp16_weights=True)
    if "token_attn" in which:
        gen_token_attn(dmh, du, mu)
    if "train" in which:
        gen_train(dmh, du, mu)
    if "dataset" in which:
        gen_dataset(du)
    for p in sorted(HERE.glob("*.npz")):
        print(p.name, p.stat().st_size)


if __name__ == "__main__":
    main()
