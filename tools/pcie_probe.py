#!/usr/bin/env python3
"""Host <-> device legs of the drop-in API at MIND-large-dev size:
which way of moving the CSR index arrays up and the scores down is fastest on
this box.  One JSON line per variant (GB/s, ms), medians of 5.

  h2d  pageable    torch.as_tensor(np).to(dev)             (the round-5 path)
       pinned      np.copyto into a cached pinned tensor, then one async copy
       (round 6 also measured a chunked, multi-threaded pinned staging ring in the
       library, nr_copy_h2d / nr_copy_d2h: 45 / 40 GB/s, slower than torch's
       pageable upload and pinned download, so it was removed; results in
       profiles/round6/pcie_probe.jsonl)
  d2h  pageable    t.cpu()
       pinned      copy_ into a pinned tensor (non_blocking) + sync
  host group_items (376 k object arrays) vs np.split

    python tools/pcie_probe.py
"""
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))


def _t(fn, reps=5):
    out = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        out.append(time.perf_counter() - t0)
    return float(np.median(out))


def main():
    from news_recommendation_project_v2_amd import ops, synthetic
    from news_recommendation_project_v2_amd.data_utils import group_items
    dev = torch.device("cuda", 0)
    n_news, n_imp = synthetic.SHAPES["mind_large_dev"]
    im = synthetic.mind_impressions(n_news, n_imp, seed=1234)
    arrs = {"hist_idx": np.ascontiguousarray(im.hist_idx, dtype=np.int32),
            "cand_idx": np.ascontiguousarray(im.cand_idx, dtype=np.int32)}
    nbytes = sum(a.nbytes for a in arrs.values())
    table = torch.randn(n_news, 1024)
    res = []

    def rec(leg, how, sec, nb):
        r = {"leg": leg, "how": how, "ms": round(sec * 1e3, 3), "GBs": round(nb / sec / 1e9, 2), "bytes": nb}
        print(json.dumps(r), flush=True)
        res.append(r)

    rec("h2d_index", "pageable", _t(lambda: [torch.as_tensor(a).to(dev) for a in arrs.values()]), nbytes)
    pins = {k: torch.empty(a.shape, dtype=torch.int32, pin_memory=True) for k, a in arrs.items()}
    rec("h2d_index", "pinned_cached (copyto + dma)",
        _t(lambda: [np.copyto(pins[k].numpy(), a) or pins[k].to(dev, non_blocking=True) for k, a in arrs.items()]),
        nbytes)
    rec("h2d_index", "pinned_dma_only", _t(lambda: [p.to(dev, non_blocking=True) for p in pins.values()]), nbytes)
    rec("h2d_index", "pinned_fresh_alloc (alloc + copyto + dma)",
        _t(lambda: [torch.from_numpy(a).pin_memory().to(dev, non_blocking=True) for a in arrs.values()]), nbytes)
    if hasattr(ops, "h2d"):
        dst = {k: torch.empty(a.shape, dtype=torch.int32, device=dev) for k, a in arrs.items()}
        rec("h2d_index", "staged (ops.h2d)", _t(lambda: [ops.h2d(dst[k], a) for k, a in arrs.items()]), nbytes)
        tdst = torch.empty(table.shape, device=dev)
        rec("h2d_table", "staged (ops.h2d)", _t(lambda: ops.h2d(tdst, table.numpy())), table.numel() * 4)
    rec("h2d_table", "pageable", _t(lambda: table.to(dev)), table.numel() * 4)

    s = torch.randn(im.n_cand, device=dev)
    rec("d2h_scores", "pageable", _t(lambda: s.cpu()), s.numel() * 4)
    ps = torch.empty(s.shape, pin_memory=True)
    rec("d2h_scores", "pinned_cached", _t(lambda: ps.copy_(s, non_blocking=True)), s.numel() * 4)
    rec("d2h_scores", "pinned_fresh_alloc", _t(lambda: torch.empty(s.shape, pin_memory=True).copy_(s, non_blocking=True)),
        s.numel() * 4)
    if hasattr(ops, "d2h"):
        host = np.empty(s.numel(), dtype=np.float32)
        rec("d2h_scores", "staged (ops.d2h)", _t(lambda: ops.d2h(host, s)), s.numel() * 4)
    ranks = np.random.default_rng(0).integers(1, 30, im.n_cand)
    rec("host_group", "group_items", _t(lambda: group_items(ranks, im.cand_len), reps=3), ranks.nbytes)
    rec("host_group", "np.split", _t(lambda: np.split(ranks, np.cumsum(im.cand_len)[:-1]), reps=3), ranks.nbytes)


if __name__ == "__main__":
    main()
