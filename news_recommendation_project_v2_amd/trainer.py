"""Config-5 trainer (reference trainer.py:952-1206, ``AttentionAttentionTrainer``).

Same constructor arguments and the same epoch loop: the training set is
``FinalAttentionTrainDataset`` (balanced positive / negative pairs per
impression, re-drawn every epoch with the shared ``rng``), batches come in
DataLoader order (shuffle=False, the dataset already permutes batches), token
states are read from the sqlite store, and every batch runs one
forward + backward + clip + AdamW step — here ``train_step.FinalAttentionTrainStep``
on the MI355X instead of torch autograd.  Per epoch the mean loss (weighted by
batch rows, trainer.py:1073-1074) is appended to
``{log_dir}/train_final_history_score.jsonl`` and the two state dicts are
saved as ``{ckpt_dir}/Epoch_{i}.pt`` (locally: the Azure blob upload of
trainer.py:1172-1197 is out of scope).

The reference sizes the batch with a GPU OOM probe
(batch_size_finder.get_attention_attention_train_batch_size); here it is an
argument (HBM is not the constraint at these shapes).
"""
from __future__ import annotations

import json
import math
import sqlite3
from datetime import datetime
from pathlib import Path
from typing import Optional

import numpy as np
import torch

from .config import DEVICE
from .data_utils import FinalAttentionTrainDataset, lengths_to_offsets, train_batch_csr
from .train_step import FinalAttentionTrainStep, LatentAttentionTrainStep, TrainBatch

DEFAULT_TRAIN_BATCH = 256


class AttentionAttentionTrainer:
    def __init__(self, db_name: str, token_attention_model: torch.nn.Module, final_attention_model: torch.nn.Module,
                 train_history_rev_index: np.ndarray, train_history_len_list: np.ndarray,
                 train_news_rev_index: np.ndarray, train_impression_len_list: np.ndarray, train_labels: np.ndarray,
                 log_dir: Optional[Path] = None, token_ckpt_dir: Optional[Path] = None,
                 final_attn_ckpt_dir: Optional[Path] = None, exp_name: str = "",
                 max_neg_ratio: Optional[float] = None, max_pos_ratio: Optional[float] = None,
                 rng: Optional[np.random.Generator] = None, batch_size: int = DEFAULT_TRAIN_BATCH,
                 dtype: torch.dtype = torch.float32, lr: float = 1e-6, dropout: float = 0.1, seed: int = 1234,
                 nan_check_every: Optional[int] = None):
        if nan_check_every is not None:
            if int(nan_check_every) < 1:
                raise ValueError("nan_check_every must be >= 1")
            self.NAN_CHECK_EVERY = int(nan_check_every)
        self.rng = rng if rng is not None else np.random.default_rng(1234)
        self.log_dir = log_dir
        self.exp_name = exp_name
        self.token_ckpt_dir = token_ckpt_dir
        self.final_attn_ckpt_dir = final_attn_ckpt_dir
        self.token_attention_model = token_attention_model
        self.final_attention_model = final_attention_model
        self.train_batch_size = batch_size
        if getattr(final_attention_model, "pooler_kind", "final") == "latent":
            # BASELINE configs[4]'s pairing: token encoder + LatentAttentionModel
            self.engine = LatentAttentionTrainStep(token_attention_model, final_attention_model, dtype=dtype, lr=lr,
                                                   seed=seed, device=DEVICE)
        else:
            self.engine = FinalAttentionTrainStep(token_attention_model, final_attention_model, dtype=dtype, lr=lr,
                                                  dropout=dropout, seed=seed, device=DEVICE)
        self.train_dataset = FinalAttentionTrainDataset(
            history_rev_index=train_history_rev_index, history_len_list=train_history_len_list,
            news_rev_index=train_news_rev_index, impression_len_list=train_impression_len_list,
            labels=train_labels, batch_size=batch_size, max_neg_raio=max_neg_ratio, max_pos_ratio=max_pos_ratio,
            rng=self.rng)
        self.connection = sqlite3.connect(str(db_name))

    def device_batch(self, lo: int, hi: int) -> TrainBatch:
        rows = [self.train_dataset[i] for i in range(lo, hi)]
        last, hidx, hoff, pos, neg = train_batch_csr(self.connection, rows)
        d = DEVICE
        return TrainBatch(tok_last=last.to(d).contiguous(), hist_idx=torch.as_tensor(hidx).to(d),
                          hist_off=torch.as_tensor(hoff).to(d), pos=torch.as_tensor(pos).to(d),
                          neg=torch.as_tensor(neg).to(d))

    # batches between host checks of the device-side losses; 1 = the reference's
    # behaviour exactly (sync on every loss, stop right after the first NaN batch)
    NAN_CHECK_EVERY = 64

    def train_one_epoch(self) -> float:
        """trainer.py:1030-1117.  The reference syncs on every loss and stops the
        epoch after the first NaN batch (whose optimizer step it has already
        applied, :1069-1072).  Here losses stay on the device and are checked
        every NAN_CHECK_EVERY batches, so up to that many further steps may run
        after a NaN (``nan_check_every=1`` checks every batch, as the reference
        does, at the cost of one host sync per step).  The parameters end NaN in
        both cases (a NaN loss means NaN gradients, and the clipped AdamW step of
        that batch already makes every parameter NaN), and the epoch loss sums
        exactly the batches before the first NaN, like the reference's
        running_loss; only the optimizer / RNG step counts can differ."""
        self.token_attention_model.train()
        self.final_attention_model.train()
        running_loss, running_count = 0.0, 0
        pending: list = []
        stop = False

        def drain() -> bool:
            nonlocal running_loss, running_count
            for loss, n in pending:
                v = float(loss.item()) if not isinstance(loss, float) else loss
                if math.isnan(v):
                    print("Nan loss found. Please check")
                    return True
                running_loss += v * n
                running_count += n
            pending.clear()
            return False

        for lo, hi in self.train_dataset.batches():
            batch = self.device_batch(lo, hi)
            pending.append((self.engine.step(batch), hi - lo))
            if len(pending) >= self.NAN_CHECK_EVERY and drain():
                stop = True
                break
        if not stop:
            drain()
        self._invalidate_eval_cache()
        return running_loss / max(running_count, 1)

    def _invalidate_eval_cache(self):
        if hasattr(self.final_attention_model, "_hip_cache"):
            self.final_attention_model._hip_cache = {}

    def train(self, num_epochs: int):
        for i in range(num_epochs):
            loss = self.train_one_epoch()
            print(i + 1, loss)
            if self.log_dir:
                Path(self.log_dir).mkdir(parents=True, exist_ok=True)
                with open(Path(self.log_dir) / "train_final_history_score.jsonl", "a") as f:
                    f.write(json.dumps({"timestamp": datetime.now().isoformat(), "exp_name": self.exp_name,
                                        "epoch": i + 1, "loss": loss}) + "\n")
            for d, m in ((self.token_ckpt_dir, self.token_attention_model),
                         (self.final_attn_ckpt_dir, self.final_attention_model)):
                if d:
                    Path(d).mkdir(parents=True, exist_ok=True)
                    torch.save({k: v.detach().cpu() for k, v in m.state_dict().items()}, Path(d) / f"Epoch_{i + 1}.pt")
            self.train_dataset.reset()
        self.connection.close()


# The reference's other trainers (trainer.py:47-949) belong to the experiments
# outside the hot path: import-level placeholders only.
from .out_of_scope import placeholder_class as _oos  # noqa: E402

ClassificationModelTrainer = _oos("ClassificationModelTrainer", "trainer.py:47-214", __name__)
AttentionWeightTrainer = _oos("AttentionWeightTrainer", "trainer.py:217-436", __name__)
AttentionTrainer = _oos("AttentionTrainer", "trainer.py:439-713", __name__)
AttentionReduceTrainer = _oos("AttentionReduceTrainer", "trainer.py:716-949", __name__)
