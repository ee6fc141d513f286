#!/usr/bin/env python3
"""Which rounding of the bf16 FinalAttention config-5 step makes its gradients
drift from the f32 oracle?  (VERDICT r4 #1.)  CPU only.

One training step from the same parameters on the reference trainer's golden
batches (tests/test_train.py fixtures), the step written out by hand with the
HIP bf16 step's rounding points (bf16 weights; S, X1, X2, X, Y, P stored bf16;
dXp, dL, dY, dX, dZ2, dZ1 stored bf16; f32 sums), each group of rounding points
switchable.  Prints the relative gradient error of the slowest tensors against
oracle/train_ref.train_step (f32 autograd) per variant:
  hip-like            every rounding point on (the HIP bf16 step)
  grads f32           backward activations unrounded
  w-branch f32        X, Y, P, W4, W5 unrounded in the forward
  exact fwd, bf16 bwd forward unrounded, backward as hip-like
  S,X1,X2 bf16x2      the inputs of linear1..3 kept as hi + lo bf16 pairs (2x
                      those GEMMs' forward MFMA work), weights and the rest bf16
  +W1..W3 bf16x2      the same with W1..W3 also split (4 products: 4x)
    python tools/bf16_ablation.py [--batches 2]
"""
import argparse
import sys
from pathlib import Path

import numpy as np
import torch
import torch.nn.functional as F

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "tests")]


def bf(t):
    return t.to(torch.bfloat16).float()


def ident(t):
    return t


def bf2(t):
    hi = bf(t)
    return hi + bf(t - hi)


def step(P, tl, hg, pos, neg, grads32=False, wbranch32=False, exact_fwd=False, x2_in=False, x2_w=False):
    qa = ident if exact_fwd else bf           # forward activations
    qi = bf2 if x2_in else qa                 # the inputs of linear1..3
    qg = ident if grads32 else bf             # backward activations
    E = F.layer_norm(tl.float(), (1024,), P["ln.weight"], P["ln.bias"], 1e-12)
    idx = torch.as_tensor(np.concatenate(hg).astype(np.int64))
    lens = [len(h) for h in hg]
    B = len(hg)
    seg = torch.repeat_interleave(torch.arange(B), torch.as_tensor(lens))
    Wb = {i: bf(P[f"linear{i}.weight"]) for i in range(1, 6)}          # backward weights: bf16
    Wf = {i: (P[f"linear{i}.weight"] if exact_fwd or (wbranch32 and i >= 4) else Wb[i]) for i in range(1, 6)}
    if x2_w:
        Wf.update({i: bf2(P[f"linear{i}.weight"]) for i in (1, 2, 3)})
    b = {i: P[f"linear{i}.bias"] for i in range(1, 5)}
    S = qi(E[idx])
    X1 = qi(F.relu(S @ Wf[1].T + b[1]))
    X2 = qi(F.relu(X1 @ Wf[2].T + b[2]))
    Xf = X2 @ Wf[3].T + b[3]
    X = Xf if wbranch32 else qa(Xf)
    Y = F.relu(X @ Wf[4].T + b[4])
    Y = Y if wbranch32 else qa(Y)
    Pf = torch.exp(Y @ Wf[5].T)
    Pm = Pf if wbranch32 else qa(Pf)
    z = torch.zeros(B, 1024).index_add_(0, seg, Pm) + 1e-10
    u = torch.zeros(B, 1024).index_add_(0, seg, X * Pm) / z
    u_, E_ = u.clone().requires_grad_(True), E.clone().requires_grad_(True)
    pn = torch.as_tensor(np.concatenate([pos, neg]).astype(np.int64))
    res = F.cosine_similarity(u_.repeat(2, 1), E_[pn])
    torch.nn.MarginRankingLoss(2.0)(*torch.chunk(res, 2), torch.tensor([1.0])).backward()
    du = u_.grad
    dXp = qg(du[seg] * Pm / z[seg])
    dL = qg(du[seg] * (X - u[seg]) * Pm / z[seg])
    dYf = (dL @ Wb[5]) * (Y > 0)
    dY = qg(dYf)
    dXf = dY @ Wb[4] + dXp
    dX = qg(dXf)
    dZ2f = (dX @ Wb[3]) * (X2 > 0)
    dZ2 = qg(dZ2f)
    dZ1f = (dZ2 @ Wb[2]) * (X1 > 0)
    dZ1 = qg(dZ1f)
    return {"linear5.weight": dL.T @ Y, "linear4.weight": dY.T @ X, "linear4.bias": dYf.sum(0),
            "linear3.weight": dX.T @ X2, "linear2.weight": dZ2.T @ X1, "linear1.weight": dZ1.T @ S,
            "linear1.bias": dZ1f.sum(0)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=2)
    args = ap.parse_args()
    from test_train import _dataset, _oracle_batch, _setup
    from test_train_bf16_drift import _params
    from oracle import train_ref
    torch.set_num_threads(8)
    g, states, labels = _setup()
    ds = _dataset(g, labels)
    p0 = _params("final")
    variants = [("hip-like", {}), ("grads f32", {"grads32": True}), ("w-branch f32", {"wbranch32": True}),
                ("exact fwd, bf16 bwd", {"exact_fwd": True}), ("S,X1,X2 bf16x2", {"x2_in": True}),
                ("+W1..W3 bf16x2", {"x2_in": True, "x2_w": True})]
    for r in ds.batches()[:args.batches]:
        tl, hg, pos, neg = _oracle_batch(ds, states, *r)[:4]
        ref = train_ref.train_step(p0, tl, hg, pos, neg, do_step=False)["grads"]
        for name, kw in variants:
            G = step(p0, tl, hg, pos, neg, **kw)
            errs = {k: round(float((G[k] - ref[k]).norm() / ref[k].norm()), 4) for k in G}
            print(r, f"{name:22s}", errs, flush=True)


if __name__ == "__main__":
    main()
