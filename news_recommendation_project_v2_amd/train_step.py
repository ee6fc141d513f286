"""One training step of config 5 on the MI355X.

Replaces the body of ``AttentionAttentionTrainer.train_one_epoch``
(trainer.py:1030-1071) for one batch:

  first_res  = token_model(tok, mask)                  # = g_mlp_LN(last valid token)
  second_res = first_res[hist] * hist_mask             # padded [B, h_max, D]
  outputs    = final_attention(second_res, hist_mask)  # train mode: dropout p = 0.1
  res        = cosine(outputs.repeat(2, 1), first_res[pos ‖ neg])
  loss       = MarginRankingLoss(2)(res[:B], res[B:], 1)
  loss.backward(); clip_grad_norm_(0.5); AdamW(lr 1e-6).step()

as ONE library call per batch (``nr_final_train_step``, csrc/final_train.hip;
no autograd, no torch kernels inside the step):
  * the token model is the g_mlp LayerNorm of the U unique news' last rows;
  * FinalAttention runs once per VALID history slot (Hs = sum h_i rows packed in
    CSR order, zero-padded to a multiple of 64): the reference's padded slots
    are masked to zero weight, so they carry no gradient and skipping them is
    exact; dropout is fused into the ReLU GEMM epilogues with a counter-hash
    stream, its backward into the data-grad GEMMs (the mask is recovered from
    the saved outputs);
  * bf16: the data-grad GEMMs also write the bias gradients (f32 column sums)
    from their epilogues, and the weight-grad GEMMs read the row-major
    activations through transposed LDS reads (no transposed copies);
  * pooling forward / backward, cosine + margin loss, scatter-add of the
    history gradient and the LayerNorm-parameter reductions are HIP kernels;
    the global grad norm and AdamW (clip coefficient folded in) are two more
    launches in ``optimizer_step``.

Parameters live in ONE flat f32 buffer (master weights; the torch modules'
parameters are re-pointed at views of it, so ``state_dict()`` is always
current), with a flat bf16 mirror for the bf16 compute dtype.  Only the
parameters that receive gradients are in it — exactly the set torch's AdamW
updates (the token model's attention / g_mlp weights and attn_layernorm get no
gradient because MyLayer discards them, attention.py:193).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

from . import ops
from ._lib import NewsRecHIPError

D = 1024
H = 4096
DROP_P = 0.1
MARGIN = 2.0  # MarginRankingLoss(2), trainer.py:985


def _pad64(n: int) -> int:
    return max(64, (n + 63) // 64 * 64)


@dataclass
class TrainBatch:
    """Device-side batch: the output of ``attention_attention_train_collate_fn``
    in CSR form (data_utils.py:893-915).

    tok_last  [U, D] f32/f16  each unique news' last valid token state
    hist_idx  [Hs] int32      history slots, indices into the U rows
    hist_off  [B+1] int64     CSR offsets of the B batch rows
    pos, neg  [B] int32       positive / negative news, indices into the U rows
    """
    tok_last: torch.Tensor
    hist_idx: torch.Tensor
    hist_off: torch.Tensor
    pos: torch.Tensor
    neg: torch.Tensor

    @property
    def B(self) -> int:
        return self.pos.numel()


def _check_loss_out(t: torch.Tensor, dev) -> torch.Tensor:
    d = torch.device(dev)
    if (t.dtype != torch.float32 or t.numel() < 1 or not t.is_contiguous() or t.device.type != d.type
            or (d.index is not None and t.device.index != d.index)):
        raise NewsRecHIPError("loss_out must be a contiguous float32 tensor with >= 1 element on the step's device")
    return t


def _weights_version(step) -> tuple:
    """Version counters of everything that can write the master weights outside
    AdamW: the flat buffer and its views (``views``), and the modules' Parameters,
    whose ``.data`` was pointed at those views -- a Parameter keeps its own version
    counter through ``.data =``, so load_state_dict on a wrapped module moves only
    the Parameter's, not the flat buffer's.  AdamW (a library call through raw
    pointers) moves neither."""
    return (step.flat._version,) + tuple(p._version for p in step._mod_params)


def _refresh_mirror(step) -> None:
    """Rewrite a step's bf16 weight mirror when its master weights changed outside
    AdamW (load_state_dict on the wrapped modules, an edit through ``views``;
    ADVICE r4)."""
    v = _weights_version(step)
    if step.flat16 is not None and v != step._mirror_version:
        with torch.no_grad():
            step.flat16.copy_(step.flat)
    step._mirror_version = v


class FinalAttentionTrainStep:
    """Owns the flat parameters, AdamW state and scratch of the config-5 step."""

    def __init__(self, token_model, final_attention, dtype: torch.dtype = torch.bfloat16, lr: float = 1e-6,
                 betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.01, max_norm: float = 0.5,
                 dropout: float = DROP_P, seed: int = 1234, device=None):
        if dtype not in (torch.float32, torch.bfloat16):
            raise NewsRecHIPError("train step dtype must be float32 or bfloat16")
        layers = list(token_model.encoder.layer)
        if len(layers) != 1:
            raise NewsRecHIPError("training supports NUM_HIDDEN_LAYERS == 1 (config.py:35)")
        self.device = device or torch.device("cuda")
        self.dtype = dtype
        # CUs the persistent GEMMs spread one 256x256 tile round over (multiple of the 8 XCDs)
        self._ncu = torch.cuda.get_device_properties(self.device).multi_processor_count // 8 * 8
        self.lr, self.betas, self.eps, self.wd, self.max_norm = lr, betas, eps, weight_decay, max_norm
        self.p = dropout
        self.seed = seed
        self.step_count = 0
        self.ln = layers[0].g_mlp_layernorm
        self.ln_eps = float(self.ln.eps)
        fa = final_attention
        self.names = ["ln.weight", "ln.bias"]
        params = [self.ln.weight, self.ln.bias]
        for i in range(1, 6):
            lin = getattr(fa, f"linear{i}")
            self.names.append(f"linear{i}.weight")
            params.append(lin.weight)
            if lin.bias is not None:
                self.names.append(f"linear{i}.bias")
                params.append(lin.bias)
        sizes = [p.numel() for p in params]
        # 16-B aligned slices (64 floats) so every view is a valid GEMM operand
        offs, o = [], 0
        for n in sizes:
            offs.append(o)
            o += (n + 63) // 64 * 64
        self.n_flat = o
        dev = self.device
        self.flat = torch.zeros(o, dtype=torch.float32, device=dev)
        self.grad = torch.zeros_like(self.flat)
        self.m = torch.zeros_like(self.flat)
        self.v = torch.zeros_like(self.flat)
        self.flat16 = torch.zeros(o, dtype=torch.bfloat16, device=dev) if dtype == torch.bfloat16 else None
        self.views, self.gviews, self.cviews = {}, {}, {}
        with torch.no_grad():
            for name, prm, off, n in zip(self.names, params, offs, sizes):
                v = self.flat[off:off + n].view(prm.shape)
                v.copy_(prm.detach().to(dev, torch.float32))
                prm.data = v  # the module now reads the master weights
                self.views[name] = v
                self.gviews[name] = self.grad[off:off + n].view(prm.shape)
                self.cviews[name] = (self.flat16[off:off + n].view(prm.shape) if self.flat16 is not None else v)
            if self.flat16 is not None:
                self.flat16.copy_(self.flat)
        self.sumsq = torch.zeros(1, dtype=torch.float32, device=dev)
        self.loss = torch.zeros(1, dtype=torch.float32, device=dev)
        self._ws = {}
        self._ws_native = None
        self._users = None
        self._mod_params = list(params)  # the modules' Parameters (now views of flat)
        self._mirror_version = _weights_version(self)
        self._pmap = {"tok_g": "ln.weight", "tok_b": "ln.bias", "W5": "linear5.weight",
                      **{f"W{i}": f"linear{i}.weight" for i in range(1, 5)},
                      **{f"b{i}": f"linear{i}.bias" for i in range(1, 5)}}

    # ------------------------------------------------------------------ helpers
    def _buf(self, name: str, shape, dtype) -> torch.Tensor:
        t = self._ws.get(name)
        n = int(np.prod(shape))
        if t is None or t.numel() < n or t.dtype != dtype:
            t = torch.empty(max(n, 1), dtype=dtype, device=self.device)
            self._ws[name] = t
        return t[:n].view(shape)

    # _tail_rows / _relu_gemm: the Python driver of the split-K tail the native
    # step runs (final_train.hip main_rows / relu_gemm), kept as its test double
    # (tests/test_train.py test_gpu_split_k_tail_matches_full_gemm).
    def _tail_rows(self, M: int, N: int, K: int) -> int:
        """Rows of a bf16 GEMM that fill whole rounds of 256x256 tiles over the CUs
        (the rest, a few tiles that would hold one CU each for a full tile time,
        run as K-slices instead); M when no such split pays -- and at K <= 1024,
        where the persistent kernel's half-tile tail is the cheaper form
        (final_train.hip split_tail)."""
        if self.dtype != torch.bfloat16 or N % 256 or K % 512 or K <= 1024 or M % 256 == 0:
            return M
        ncu = self._ncu
        ntn = N // 256
        if ncu % ntn:
            return M
        m_main = M // (256 * (ncu // ntn)) * (256 * (ncu // ntn))
        tail_tiles = -(-(M - m_main) // 256) * ntn
        return m_main if m_main > 0 and tail_tiles * 4 <= ncu else M

    def _relu_gemm(self, a: torch.Tensor, w: torch.Tensor, out: torch.Tensor, *, bias=None, seed: int = 0,
                   y: Optional[torch.Tensor] = None, scale: float = 1.0) -> torch.Tensor:
        """gemm_relu_dropout (y None) or gemm_drelu (y = forward output).  When the
        last round of 256x256 tiles would be a few tiles (M just past a multiple
        of 16 M-tiles at N = 4096: M = 8,320 -> 512 + 16 tiles, the 16 costing a
        whole tile time), those rows run as 8 K-slices in one grouped launch plus
        nr_splitk_fixup (sum + bias + the same epilogue / dropout mask)."""
        M, K = a.shape
        N = w.shape[0]
        mm = self._tail_rows(M, N, K)
        if mm > 0:
            if y is None:
                ops.gemm_relu_dropout(a[:mm], w, bias, seed, self.p, out=out[:mm])
            else:
                ops.gemm_drelu(a[:mm], w, y[:mm], scale, out=out[:mm])
        if mm == M:
            return out
        parts, kk = 8, K // 8
        P = self._buf("splitk_P", (parts, M - mm, N), torch.float32)
        ops.gemm_grouped([(a[mm:, i * kk:(i + 1) * kk], w[:, i * kk:(i + 1) * kk], P[i]) for i in range(parts)])
        ops.splitk_fixup(P, out[mm:], "relu_dropout" if y is None else "drelu", bias=bias,
                         residual=None if y is None else y[mm:], row0=mm, seed=seed, p=self.p, scale=scale)
        return out

    def W(self, i: int) -> torch.Tensor:
        return self.cviews[f"linear{i}.weight"]

    def b(self, i: int) -> Optional[torch.Tensor]:
        return self.views.get(f"linear{i}.bias")

    def layer_seed(self, layer: int) -> int:
        """Dropout stream of one forward layer in the current step."""
        return (self.seed * 1_000_003 + self.step_count * 7919 + layer * 104_729) & (2**64 - 1)

    # ------------------------------------------------------------------ step
    def forward_backward(self, batch: TrainBatch, loss_out: torch.Tensor | None = None):
        """Loss (device scalar, written to ``loss_out`` when given) and gradients
        into ``self.grad`` (every slice rewritten) as ONE library call (``nr_final_train_step``, csrc/final_train.hip):
        the forward, the margin loss and the whole backward of the batch.
        Returns (loss, users, None): users = the pooled users [B, D] f32.  Both
        returned tensors are views of buffers the next call overwrites in place
        (on the stream); clone them to keep a step's values."""
        from . import _lib
        U, B, Hs = batch.tok_last.shape[0], batch.B, batch.hist_idx.numel()
        lib = _lib.load()
        self._refresh_mirror()
        dt = _lib.NR_BF16 if self.dtype == torch.bfloat16 else _lib.NR_F32
        with torch.cuda.device(self.device):
            need = int(lib.nr_final_train_workspace_bytes(dt, B, U, Hs))
        if self._ws_native is None or self._ws_native.numel() < need:
            self._ws_native = torch.empty(need, dtype=torch.uint8, device=self.device)
        if self._users is None or self._users.shape[0] < B:
            self._users = torch.empty((B, D), dtype=torch.float32, device=self.device)
        tok = batch.tok_last.contiguous()
        tdt = {torch.float32: _lib.NR_F32, torch.bfloat16: _lib.NR_BF16, torch.float16: _lib.NR_F16}[tok.dtype]
        hi, ho = batch.hist_idx.to(torch.int32).contiguous(), batch.hist_off.to(torch.int64).contiguous()
        pos, neg = batch.pos.to(torch.int32).contiguous(), batch.neg.to(torch.int32).contiguous()
        a = _lib.FinalTrainArgs()
        a.dtype, a.tok_dtype, a.B, a.U, a.Hs, a.margin, a.p = dt, tdt, B, U, Hs, MARGIN, self.p
        for i in range(3):
            a.seed[i] = self.layer_seed(i + 1)
        a.tok_last, a.hist_idx, a.hist_off, a.pos, a.neg = (tok.data_ptr(), hi.data_ptr(), ho.data_ptr(), pos.data_ptr(),
                                                            neg.data_ptr())
        for f, name in self._pmap.items():
            src = self.cviews[name] if f.startswith("W") else self.views[name]
            setattr(a, f, src.data_ptr())
            setattr(a, "g_" + f, self.gviews[name].data_ptr())
        loss = self.loss if loss_out is None else _check_loss_out(loss_out, self.device)
        a.loss, a.users, a.sumsq = loss.data_ptr(), self._users.data_ptr(), self.sumsq.data_ptr()
        _lib.check(lib.nr_final_train_step(ctypes.byref(a), self._ws_native.data_ptr(), self._ws_native.numel(),
                                           torch.cuda.current_stream(self.device).cuda_stream), "nr_final_train_step")
        self._keep = (tok, hi, ho, pos, neg)  # alive until the stream has run the step
        return loss, self._users[:B], None

    def _refresh_mirror(self) -> None:
        _refresh_mirror(self)

    def optimizer_step(self) -> None:
        """clip_grad_norm_(max_norm) + AdamW (trainer.py:1067-1069): one launch; the
        squared grad norm was summed by the step itself (``sumsq``)."""
        self.step_count += 1
        ops.adamw(self.flat, self.grad, self.m, self.v, self.step_count, self.lr, self.betas, self.eps, self.wd,
                  self.max_norm, self.sumsq if self.max_norm > 0 else None, self.flat16)

    def step(self, batch: TrainBatch) -> torch.Tensor:
        """One full step; returns this step's loss as its own device scalar (a
        fresh allocation the step writes, so no copy launch)."""
        out = torch.empty(1, dtype=torch.float32, device=self.device)
        self.forward_backward(batch, loss_out=out)
        self.optimizer_step()
        return out

    def grad_dict(self) -> dict:
        return {k: v for k, v in self.gviews.items()}

    def flops_per_step(self, Hs: int) -> float:
        """MFMA FLOPs of one step (forward + data-grad + weight-grad GEMMs)."""
        Hp = _pad64(Hs)
        fwd = 2.0 * Hp * (D * H + H * H + H * D + D * H + H * D)
        return 3.0 * fwd

    def hbm_bytes_per_step(self, Hs: int, U: int) -> dict:
        """Algorithmic HBM bytes of the step's non-GEMM kernels (the GEMMs are
        priced by their FLOPs): AdamW 30 B per parameter (f32 param, grad, m, v
        read; param, m, v written; the bf16 mirror written) and the row kernels
        per history slot (es = 2 bf16): slots_kernel reads the token row and
        writes S and XH (2 D es), pool fwd reads (X, P) (2 D es), pool bwd reads
        them again and writes dXp and dL (4 D es) -- 8 D es per slot -- plus the
        four weight transposes read and written once (W5, W4, W3: D H each;
        W2: H H)."""
        es = 2 if self.dtype == torch.bfloat16 else 4
        Hp = _pad64(Hs)
        rows = Hp * 8 * D * es + U * D * 2 + 2 * es * (3 * D * H + H * H)
        return {"adamw": 30.0 * self.n_flat, "row_kernels": float(rows)}


class LatentAttentionTrainStep:
    """Config-5 step with ``LatentAttentionModel`` in the pooler slot (BASELINE
    configs[4]: "backward for encoder + latent attention"; the reference
    trainer's loop, trainer.py:1044-1069, with the latent pooler) as ONE library
    call per batch (``nr_latent_train_step``, csrc/latent_train.hip):

      E     = g_mlp_LN(last token of each unique news)
      fold  K/V of the 64 latents into A (scores) and Bt (output) once per step
      per history slot: X = LN_q(E[hist]); P = softmax64(X Aᵀ); H1 = P Btᵀ + E[hist];
                        Z = GEGLU(LN_f(H1) W1ᵀ + b1)
      per batch row:    m = mean(Z) W2ᵀ + b2 + mean(H1)  (the last linear layer commutes
                        with the history mean: its three GEMMs run over B rows, not slots)
      users = normalize(m); loss = MarginRankingLoss(2)(cos(users, E[pos]), cos(users, E[neg]))
      backward of all of it; clip_grad_norm_(0.5) + AdamW   (grad norm in the step), nr_adamw

    dtype float32: exact-f32 MFMA GEMMs and f32 activations (the parity mode);
    bfloat16: bf16 operands and activations with f32 accumulation, statistics
    and gradients, weights read from a bf16 mirror AdamW rewrites.  The
    parameters are views of one flat f32 buffer (as in FinalAttentionTrainStep),
    so ``state_dict()`` stays current and AdamW is one launch."""

    def __init__(self, token_model, latent_model, dtype: torch.dtype = torch.float32, lr: float = 1e-6,
                 betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.01, max_norm: float = 0.5,
                 seed: int = 1234, device=None):
        # (no dropout argument: LatentAttentionModel has no dropout, latent_attention.py:77-171)
        if dtype not in (torch.float32, torch.bfloat16):
            raise NewsRecHIPError("latent-attention train step dtype must be float32 or bfloat16")
        layers = list(token_model.encoder.layer)
        if len(layers) != 1:
            raise NewsRecHIPError("training supports NUM_HIDDEN_LAYERS == 1 (config.py:35)")
        self.device = device or torch.device("cuda")
        self.dtype = dtype
        self.lr, self.betas, self.eps, self.wd, self.max_norm = lr, betas, eps, weight_decay, max_norm
        self.seed = seed
        self.step_count = 0
        self.ln = layers[0].g_mlp_layernorm
        self.ln_eps = float(self.ln.eps)
        if abs(self.ln_eps - 1e-12) > 1e-18:
            raise NewsRecHIPError("the token LayerNorm of MyLayer has eps 1e-12 (attention.py:155)")
        self.model = latent_model
        lat = list(latent_model.named_parameters())
        self.names = ["ln.weight", "ln.bias"] + [f"latent.{n}" for n, _ in lat]
        params = [self.ln.weight, self.ln.bias] + [p for _, p in lat]
        offs, o = [], 0
        for prm in params:
            offs.append(o)
            o += (prm.numel() + 63) // 64 * 64
        dev = self.device
        self.n_flat = o
        self.flat = torch.zeros(o, dtype=torch.float32, device=dev)
        self.grad = torch.zeros_like(self.flat)
        self.m = torch.zeros_like(self.flat)
        self.v = torch.zeros_like(self.flat)
        self.flat16 = torch.zeros(o, dtype=torch.bfloat16, device=dev) if dtype == torch.bfloat16 else None
        self.views, self.gviews, self.cviews = {}, {}, {}
        with torch.no_grad():
            for name, prm, off in zip(self.names, params, offs):
                n = prm.numel()
                view = self.flat[off:off + n].view(prm.shape)
                view.copy_(prm.detach().to(dev, torch.float32))
                prm.data = view  # the modules now read the master weights
                self.views[name] = view
                self.gviews[name] = self.grad[off:off + n].view(prm.shape)
                self.cviews[name] = self.flat16[off:off + n].view(prm.shape) if self.flat16 is not None else view
            if self.flat16 is not None:
                self.flat16.copy_(self.flat)
        self.sumsq = torch.zeros(1, dtype=torch.float32, device=dev)
        self.loss = torch.zeros(1, dtype=torch.float32, device=dev)
        self._ws = None
        self._users = None
        self._mod_params = list(params)  # the modules' Parameters (now views of flat)
        self._mirror_version = _weights_version(self)
        b = "latent.cross_attend_blocks."
        self._pmap = {"tok_g": "ln.weight", "tok_b": "ln.bias", "latents": "latent.latents",
                      "nq_g": b + "0.norm.weight", "nq_b": b + "0.norm.bias",
                      "nc_g": b + "0.norm_context.weight", "nc_b": b + "0.norm_context.bias",
                      "Wq": b + "0.fn.to_q.weight", "Wkv": b + "0.fn.to_kv.weight", "Wo": b + "0.fn.to_out.weight",
                      "nf_g": b + "1.norm.weight", "nf_b": b + "1.norm.bias",
                      "W1": b + "1.fn.net.0.weight", "b1": b + "1.fn.net.0.bias",
                      "W2": b + "1.fn.net.2.weight", "b2": b + "1.fn.net.2.bias"}
        if set(self._pmap.values()) != set(self.names):
            raise NewsRecHIPError(f"unexpected LatentAttentionModel parameters: {sorted(self.names)}")

    def forward_backward(self, batch: TrainBatch, loss_out: torch.Tensor | None = None):
        """Loss (device scalar, written to ``loss_out`` when given) and gradients
        into ``self.grad`` (every slice rewritten).  Returns (loss, users, None): users = the normalized pooled
        users [B, D].  Both are views of buffers the next call overwrites in
        place (on the stream); clone them to keep a step's values."""
        from . import _lib
        U, B, Hs = batch.tok_last.shape[0], batch.B, batch.hist_idx.numel()
        lib = _lib.load()
        _refresh_mirror(self)
        dt = _lib.NR_BF16 if self.dtype == torch.bfloat16 else _lib.NR_F32
        need = int(lib.nr_latent_train_workspace_bytes(dt, B, U, Hs))
        if self._ws is None or self._ws.numel() < need:
            self._ws = torch.empty(need, dtype=torch.uint8, device=self.device)
        if self._users is None or self._users.shape[0] < B:
            self._users = torch.empty((B, D), dtype=torch.float32, device=self.device)
        tok = batch.tok_last.contiguous()
        tdt = {torch.float32: _lib.NR_F32, torch.bfloat16: _lib.NR_BF16, torch.float16: _lib.NR_F16}[tok.dtype]
        hi, ho = batch.hist_idx.to(torch.int32).contiguous(), batch.hist_off.to(torch.int64).contiguous()
        pos, neg = batch.pos.to(torch.int32).contiguous(), batch.neg.to(torch.int32).contiguous()
        a = _lib.LatentTrainArgs()
        a.dtype, a.tok_dtype, a.B, a.U, a.Hs, a.margin = dt, tdt, B, U, Hs, MARGIN
        a.tok_last, a.hist_idx, a.hist_off, a.pos, a.neg = (tok.data_ptr(), hi.data_ptr(), ho.data_ptr(), pos.data_ptr(),
                                                            neg.data_ptr())
        for f, name in self._pmap.items():
            src = self.cviews[name] if f in ("Wq", "Wkv", "Wo", "W1", "W2") else self.views[name]
            setattr(a, f, src.data_ptr())
            setattr(a, "g_" + f, self.gviews[name].data_ptr())
        loss = self.loss if loss_out is None else _check_loss_out(loss_out, self.device)
        a.loss, a.users, a.sumsq = loss.data_ptr(), self._users.data_ptr(), self.sumsq.data_ptr()
        # (no grad.zero_(): the step writes every gradient and zeroes its own accumulators;
        # the flat buffer's alignment gaps were zeroed at construction and are never written)
        _lib.check(lib.nr_latent_train_step(ctypes.byref(a), self._ws.data_ptr(), self._ws.numel(),
                                            torch.cuda.current_stream(self.device).cuda_stream),
                   "nr_latent_train_step")
        self._keep = (tok, hi, ho, pos, neg)  # alive until the stream has run the step
        return loss, self._users[:B], None

    def optimizer_step(self) -> None:
        """clip_grad_norm_(max_norm) + AdamW in one launch (trainer.py:1067-1069): the
        squared grad norm was summed by the step itself (``sumsq``, each stream over
        the gradients it wrote); the bf16 mode's weight mirror is rewritten by the
        same AdamW launch."""
        self.step_count += 1
        ops.adamw(self.flat, self.grad, self.m, self.v, self.step_count, self.lr, self.betas, self.eps, self.wd,
                  self.max_norm, self.sumsq if self.max_norm > 0 else None, self.flat16)
        if hasattr(self.model, "_hip_cache"):
            self.model._hip_cache = {}  # the eval path's folded weights are stale now

    def step(self, batch: TrainBatch) -> torch.Tensor:
        out = torch.empty(1, dtype=torch.float32, device=self.device)
        self.forward_backward(batch, loss_out=out)
        self.optimizer_step()
        return out

    def grad_dict(self) -> dict:
        return dict(self.gviews)

    def flops_per_step(self, Hs: int, B: int = 256) -> float:
        """MFMA FLOPs the step executes (forward, data-grad and weight-grad GEMMs,
        the fold and its backward; the last layer's GEMMs over B rows)."""
        Hp, Bp = _pad64(Hs), _pad64(B)
        slot = 2.0 * Hp * (D * 512 + 512 * D + D * 8192)          # P, H1, G
        row = 2.0 * Bp * 4096 * D                                  # m = mean(Z) W2^T
        fold = 2.0 * 64 * D * 8192 + 2 * (2.0 * 8 * 64 * 512 * D)  # KV, A, Bt^T
        return 3.0 * (slot + row + fold)

    def hbm_bytes_per_step(self, Hs: int, U: int) -> dict:
        """Algorithmic HBM bytes of the step's non-GEMM kernels (the GEMMs are
        priced by their FLOPs): AdamW 30 B per parameter (f32 param, grad, m, v
        read; param, m, v written; the bf16 mirror written) and the row kernels
        per history slot (es = 2 bf16): gather + LN_q writes S and X (2 D es);
        segmean reads G and H1 (8192 es + D es); the GEGLU backward reads G and
        writes dG (2 x 8192 es); the LN_f backward reads H1 and dY and writes dH1
        (3 D es); the LN_q backward reads dX and X and adds dE in f32 (2 D es +
        4 D) -- 32,768 es + 4 D bytes per slot -- plus the token rows read."""
        es = 2 if self.dtype == torch.bfloat16 else 4
        Hp = _pad64(Hs)
        per_slot = (2 * D + 8192 + D + 2 * 8192 + 3 * D + 2 * D) * es + 4 * D
        return {"adamw": 30.0 * self.n_flat, "row_kernels": float(Hp * per_slot + U * D * 2)}

    def model_flops_per_step(self, Hs: int) -> float:
        """The reference formulation's GEMM FLOPs (every linear layer per history
        slot, K/V once): what rounds 1-3 reported as this step's gemm_tflops."""
        Hp = _pad64(Hs)
        return 3.0 * 2.0 * Hp * (D * 512 + 512 * D + D * 8192 + 4096 * D)
