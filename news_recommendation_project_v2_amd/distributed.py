"""Multi-GPU eval: one process per GPU, torch.distributed over RCCL (xGMI).

The reference has no distributed code; this is the one
parallel strategy the hot path needs:
  phase A  each rank runs the per-news pooler transform on a contiguous
           1/world slice of the news table (MFMA GEMMs, no communication);
  phase B  the all-gather of the [N/world, k*1024] slices (RCCL ncclAllGather
           over xGMI) gives every GPU the full table (opt-in: the shard is
           transformed in chunks and chunk c's all-gather overlaps chunk c+1's
           transform);
  phase C  impressions are split into contiguous, cost-balanced ranges and
           pooled + scored with no further communication.
Scores stay on their rank; ``gather_scores`` concatenates them in impression
order on rank 0 when the caller wants them on the host.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch
import torch.distributed as dist

from .engine import PoolScoreEngine


def _host_staged(group=None) -> bool:
    """True for gloo, which moves host buffers: device tensors are staged through
    the host.  (RCCL needs one GPU per rank; the multi-rank GPU test runs gloo
    ranks that share the box's one GPU.)"""
    return dist.get_backend(group) == "gloo"


def shard_rows(n: int, world: int) -> int:
    """Rows per rank for the news-table shard (ceil), so all shards are equal."""
    return (n + world - 1) // world


def partition_by_cost(hist_len: np.ndarray, cand_len: np.ndarray, world: int, table_row_bytes: int,
                      cand_row_bytes: int) -> np.ndarray:
    """Contiguous impression ranges balanced by the prefix sum of
    cost_i = c_i*(cand_row_bytes + 8) + h_i*(table_row_bytes + 4)  (SURVEY §8(e)).
    Returns ``world + 1`` boundaries."""
    cost = cand_len.astype(np.float64) * (cand_row_bytes + 8) + hist_len.astype(np.float64) * (table_row_bytes + 4)
    cs = np.concatenate([[0.0], np.cumsum(cost)])
    targets = cs[-1] * np.arange(world + 1) / world
    b = np.searchsorted(cs, targets, side="left")
    b[0], b[-1] = 0, len(hist_len)
    return np.maximum.accumulate(b).astype(np.int64)


class NrComm:
    """The library's own RCCL communicator (include/newsrec.h nr_comm_*,
    SURVEY §8(b) nr_allgather): rank 0 draws the 128-byte unique id
    (nr_comm_unique_id), the host broadcasts it over the torch.distributed
    group, and every rank joins (nr_comm_init, collective).  ``allgather``
    issues ncclAllGather on the current torch stream."""

    def __init__(self, rank: int, world: int, group=None, timeout_s: float = 300.0):
        """Collective over the group: every rank returns, or every rank raises.
        A failure on one rank is agreed on before the next collective step (a
        status byte travels with the id; a MIN all-reduce of a ready flag
        precedes nr_comm_init and one of a success flag follows it), so no rank
        is left waiting in a collective its peers have abandoned.  A rank dying
        INSIDE the RCCL init after the ready check is covered by the deadline:
        the communicator is formed non-blocking (nr_comm_init_timeout) and
        aborted after ``timeout_s`` (NR_ERR_TIMEOUT on the surviving ranks)
        instead of blocking them forever; ``timeout_s <= 0``
        is the blocking init."""
        import ctypes
        from . import _lib
        self.rank, self.world = rank, world
        self._h = ctypes.c_void_p()
        flag_dev = "cpu" if _host_staged(group) else torch.device("cuda", torch.cuda.current_device())
        buf = (ctypes.c_ubyte * (1 + 128))()
        err = None
        try:
            self._lib = _lib.load()
            if rank == 0:
                _lib.check(self._lib.nr_comm_unique_id(ctypes.cast(ctypes.byref(buf, 1),
                                                                   ctypes.POINTER(ctypes.c_ubyte))),
                           "nr_comm_unique_id")
                buf[0] = 1
        except Exception as e:  # noqa: BLE001  (reported on every rank below)
            err = e
        t_id = torch.tensor(list(buf), dtype=torch.uint8, device=flag_dev)
        dist.broadcast(t_id, src=0, group=group)
        if int(t_id[0].item()) != 1:
            raise RuntimeError(f"NrComm: rank 0 could not create the RCCL unique id ({err!r})")
        idb = (ctypes.c_ubyte * 128)(*t_id[1:].cpu().tolist())
        try:
            if err is None:
                _lib.check(self._lib.nr_init(torch.cuda.current_device()), "nr_init")
        except Exception as e:  # noqa: BLE001
            err = e
        self._agree(err is None, group, flag_dev, "before nr_comm_init", err)
        try:
            _lib.check(self._lib.nr_comm_init_timeout(ctypes.byref(self._h), idb, world, rank,
                                                      int(timeout_s * 1000) if timeout_s > 0 else 0),
                       "nr_comm_init_timeout")
        except Exception as e:  # noqa: BLE001
            err = e
        try:
            self._agree(err is None, group, flag_dev, "in nr_comm_init", err)
        except RuntimeError:
            self.close()
            raise

    def _agree(self, ok: bool, group, flag_dev, where: str, err) -> None:
        """MIN all-reduce of this rank's flag: raise on every rank if any failed."""
        t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=flag_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
        if int(t.item()) != 1:
            raise RuntimeError(f"NrComm: a rank failed {where} (this rank: {err!r})")

    def allgather(self, send: torch.Tensor, recv: torch.Tensor) -> None:
        from . import _lib
        nb = send.numel() * send.element_size()
        assert recv.numel() * recv.element_size() == nb * self.world and send.is_contiguous() and recv.is_contiguous()
        _lib.check(self._lib.nr_allgather(self._h, send.data_ptr(), recv.data_ptr(), nb,
                                          torch.cuda.current_stream().cuda_stream), "nr_allgather")

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.nr_comm_destroy(self._h)
            self._h = None

    def __del__(self):  # best effort; call close() explicitly before the process group goes
        try:
            self.close()
        except Exception:
            pass


# the shard's transform is cut in two (rows permitting) so that the all-gather of
# the first half runs on the communicator's stream while the second half is
# transformed.  Measured price of the cut alone (tools/chunk_probe.py, latent
# bf16, profiles/round2/overlap/chunks.jsonl): +0.07 ms at 36 k shard rows
# (N = 2), +0.05 at 18 k (N = 4), +0.19 at 9 k (N = 8, where the chain's
# K = 4096 GEMM is one tile round either way) -- against half of the
# all-gather (74 / 110 / 129 MB inbound per GPU at N = 2 / 4 / 8 over 1 / 3 /
# 7 xGMI links).  Whether RCCL's kernels actually run beside the persistent GEMMs
# at world > 1 (and whether RCCL_CUS is enough) has not been measured on a
# multi-GPU node yet, so the overlap is opt-in (``chunks="auto"`` or an int); the
# default is one transform + one in-place all_gather_into_tensor.  The bench at
# N > 1 measures both and checks the tables agree bit for bit.
CHUNK_MIN_ROWS = 8192
# CUs left to RCCL's kernels while the persistent GEMMs of an overlapped chunk
# run (a persistent GEMM workgroup holds a whole CU)
RCCL_CUS = 16


class ShardedTable:
    """Phase A + B: sharded per-news transform and the one-time all-gather.

    Default (``chunks=1``): the shard is transformed, then one in-place
    all_gather_into_tensor.  With ``chunks`` > 1 (or "auto": 2 at world > 1
    when each half has at least CHUNK_MIN_ROWS rows) the shard's rows are
    transformed chunk by chunk and each chunk is all-gathered asynchronously
    (``dist.all_gather`` into the rank-major table's row ranges) while the next
    chunk is transformed; the persistent GEMMs of the chunks then run on all but
    RCCL_CUS CUs.

    ``timing=True`` records HIP events on the current stream around the
    transform and around the collective (chunks == 1: the current stream waits
    for RCCL's stream at the end of the call, so the second interval is the
    all-gather); ``last_ms()`` reads them after a sync."""

    def __init__(self, engine: PoolScoreEngine, rank: int, world: int, group=None, chunks=1, timing: bool = False,
                 comm: Optional[NrComm] = None):
        self.eng, self.rank, self.world, self.group = engine, rank, world, group
        # comm: run the all-gather through the library's own RCCL communicator
        # (nr_allgather) instead of torch.distributed's (one chunk only)
        self.comm = comm
        n = engine.hist_src.shape[0]
        self.rows = shard_rows(n, world)
        width = 2048 if engine.pooler == "final" else 1024
        # the engine's source table is left as it is; when N is not a multiple of
        # world the LAST rank's slice is short and it transforms a zero-padded copy
        # of just that slice (every rank contributes `rows` rows to the gather)
        self.src = engine.hist_src
        lo, hi = rank * self.rows, min((rank + 1) * self.rows, n)
        self.lo = lo
        if hi - lo != self.rows:
            part = torch.zeros((self.rows, engine.hist_src.shape[1]), dtype=engine.hist_src.dtype,
                               device=engine.device)
            if hi > lo:
                part[:hi - lo] = engine.hist_src[lo:hi]
            self.src, self.lo = part.contiguous(), 0
        self.full = torch.empty((self.rows * world, width), dtype=engine.dtype, device=engine.device)
        # RCCL all-gathers in place (the rank's input is its own slice of the output);
        # gloo needs a separate host-staged input
        in_place = world == 1 or not _host_staged(group)
        self.local = self.full[rank * self.rows:(rank + 1) * self.rows] if in_place else \
            torch.empty((self.rows, width), dtype=engine.dtype, device=engine.device)
        if chunks is None or chunks == "auto":
            chunks = 2 if world > 1 and self.rows >= 2 * CHUNK_MIN_ROWS and comm is None else 1
        if comm is not None and chunks != 1:
            raise ValueError("ShardedTable: the nr_allgather path gathers the shard in one piece (chunks=1)")
        self.chunks = max(1, min(int(chunks), self.rows))
        self.bounds = [round(c * self.rows / self.chunks) for c in range(self.chunks + 1)]
        self.timing = bool(timing) and self.full.is_cuda
        self._ev = None

    def _mark(self, i: int) -> None:
        if self.timing:
            if self._ev is None:
                self._ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            self._ev[i].record()

    def last_ms(self):
        """(transform_ms, allgather_ms) of the last build() with timing on (the
        all-gather interval includes any wait for the collective); None for the
        overlapped path's gather, which has no separate interval."""
        if not self._ev:
            return None
        t = self._ev[0].elapsed_time(self._ev[1])
        g = self._ev[1].elapsed_time(self._ev[2]) if self.chunks == 1 else None
        return t, g

    @property
    def gather_bytes_in(self) -> int:
        """Bytes each rank receives from its peers in the all-gather."""
        return (self.world - 1) * self.rows * self.full.shape[1] * self.full.element_size()

    def _overlapped(self) -> None:
        """Transform chunk c, then all-gather it asynchronously (byte views: any
        dtype, any backend) while chunk c + 1 is transformed.  One chunk: the
        in-place all_gather_into_tensor (no staging buffer, no copies)."""
        from . import ops
        if self.chunks == 1:
            self._mark(0)
            self.eng.transform(rows=slice(self.lo, self.lo + self.rows), out=self.local, src=self.src)
            self._mark(1)
            if self.comm is not None:
                self.comm.allgather(self.local.view(torch.uint8), self.full.view(torch.uint8))
            else:
                dist.all_gather_into_tensor(self.full.view(torch.uint8), self.local.view(torch.uint8), group=self.group)
            self._mark(2)
            return
        reserve = self.full.is_cuda and self.chunks > 1
        prev = ops.persistent_workgroups() if reserve else 0
        if reserve:
            ncu = torch.cuda.get_device_properties(self.full.device).multi_processor_count
            ops.set_persistent_workgroups(max(8, (ncu - RCCL_CUS) // 8 * 8))
        works = []
        self._mark(0)
        try:
            for a, b in zip(self.bounds[:-1], self.bounds[1:]):
                self.eng.transform(rows=slice(self.lo + a, self.lo + b), out=self.local[a:b], src=self.src)
                outs = [self.full[r * self.rows + a:r * self.rows + b].view(torch.uint8) for r in range(self.world)]
                works.append(dist.all_gather(outs, self.local[a:b].view(torch.uint8), group=self.group, async_op=True))
        finally:
            if reserve:
                ops.set_persistent_workgroups(prev)
            # every collective already issued completes before this rank leaves (on an
            # exception too: peers are inside the same collectives and would hang)
            for w in works:
                w.wait()
        self._mark(1)
        self._mark(2)

    def build(self) -> torch.Tensor:
        if self.comm is not None or (self.world > 1 and not (_host_staged(self.group) and self.local.is_cuda)):
            self._overlapped()
            self.eng.hist_table = self.full
            return self.full
        self._mark(0)
        self.eng.transform(rows=slice(self.lo, self.lo + self.rows), out=self.local, src=self.src)
        self._mark(1)
        if self.world > 1:
            if _host_staged(self.group) and self.local.is_cuda:
                # gloo moves host memory: stage the slices through the host as raw bytes
                host = torch.empty(self.full.shape, dtype=self.full.dtype)
                dist.all_gather_into_tensor(host.view(torch.uint8), self.local.cpu().view(torch.uint8),
                                            group=self.group)
                self.full.copy_(host)
        self._mark(2)
        self.eng.hist_table = self.full
        return self.full


def sharded_step(table: ShardedTable, want_users: bool = False, scores: Optional[torch.Tensor] = None):
    """One eval pass on this rank: A + B (table), inverse norms, C (pool+score)."""
    table.build()
    table.eng.inv_norms()
    return table.eng.pool_score(want_users=want_users, scores=scores)


def gather_scores(local_scores: torch.Tensor, world: int, group=None) -> Optional[torch.Tensor]:
    """Concatenate per-rank score vectors (impression order) on every rank."""
    if world == 1:
        return local_scores
    if _host_staged(group) and local_scores.is_cuda:
        return gather_scores(local_scores.cpu(), world, group).to(local_scores.device)
    n = torch.tensor([local_scores.numel()], device=local_scores.device, dtype=torch.int64)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    m = int(max(int(s) for s in sizes))
    buf = torch.zeros(m, dtype=local_scores.dtype, device=local_scores.device)
    buf[:local_scores.numel()] = local_scores
    outs = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(outs, buf, group=group)
    return torch.cat([o[:int(s)] for o, s in zip(outs, sizes)])


def sharded_second_attention_score(history_rev_index, history_len_list, news_rev_index, impression_len_list,
                                   news_embeddings: torch.Tensor, history_bool, attention_model: torch.nn.Module,
                                   dtype: Optional[torch.dtype], rank: int, world: int, group=None) -> dict:
    """``get_final_second_attention_score`` (data_model_helper.py:416-443) over
    ``world`` ranks, one GPU each (BASELINE config 4): the impressions that have a
    history are split into contiguous cost-balanced ranges (``partition_by_cost``),
    every rank transforms 1/world of the news table and all-gathers it (RCCL),
    pools + scores its own range, and the scores are gathered back in impression
    order on every rank, where the dense ranks are taken exactly as on one GPU.
    Same return value as the single-GPU function (bit-identical scores: every
    row and impression is computed by the same kernels)."""
    from . import ops
    from .data_model_helper import COMPUTE_DTYPE
    from .data_utils import group_items, lengths_to_offsets, rank_group_preds
    dtype = dtype or COMPUTE_DTYPE
    hb = np.asarray(history_bool, dtype=bool)
    imp_len = np.asarray(impression_len_list)
    sub_news = np.asarray(news_rev_index)[np.repeat(hb, imp_len)]
    sub_len = imp_len[hb]
    hist_idx = np.asarray(history_rev_index)
    hist_len = np.asarray(history_len_list)
    assert len(hist_len) == len(sub_len), "Number of rows should be consistent"
    es = 2 if dtype == torch.bfloat16 else 4
    k = 2 if attention_model.pooler_kind == "final" else 1
    b = partition_by_cost(hist_len, sub_len, world, k * 1024 * es, 1024 * es)
    a, e = int(b[rank]), int(b[rank + 1])
    ho, co = lengths_to_offsets(hist_len), lengths_to_offsets(sub_len)
    dev = torch.device("cuda", torch.cuda.current_device())
    eng = PoolScoreEngine(attention_model, dtype=dtype, device=dev).load_news(news_embeddings)
    eng.load_impressions(hist_idx[ho[a]:ho[e]], hist_len[a:e], sub_news[co[a]:co[e]], sub_len[a:e])
    local, _ = sharded_step(ShardedTable(eng, rank, world, group))
    scores_d = gather_scores(local, world, group)
    scores = scores_d.cpu().numpy()
    if hb.all():
        off = torch.as_tensor(lengths_to_offsets(imp_len)).to(dev)
        grouped = group_items(ops.dense_rank(scores_d.contiguous(), off).cpu().numpy().astype(np.int64), imp_len)
    else:  # reference quirk: grouping by the unfiltered lengths (see get_final_second_attention_score)
        grouped = rank_group_preds(scores, imp_len)
    return {"scores": scores, "grouped_scores": grouped}
