"""World-size-2 gloo tests of the multi-GPU plumbing on the CPU: news-table
sharding + padding + all-gather, score gathering, cost-balanced impression
partitioning.  The per-news transform is stubbed with a deterministic CPU
function (the HIP transform is covered by the GPU tests)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from news_recommendation_project_v2_amd.distributed import (ShardedTable, gather_scores, partition_by_cost,
                                                             shard_rows)


class StubEngine:
    """Engine stand-in: transform(rows) = 2*rows + 1 (k=1 layout)."""

    pooler = "latent"

    def __init__(self, table):
        self.hist_src = table
        self.dtype = table.dtype
        self.device = table.device
        self.hist_table = None

    def transform(self, rows=None, out=None, src=None):
        src = self.hist_src if src is None else src
        src = src if rows is None else src[rows]
        res = src * 2 + 1
        if out is not None:
            out.copy_(res)
            return out
        return res


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_news, q, chunks=None):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        table = torch.arange(n_news * 1024, dtype=torch.float32).reshape(n_news, 1024) / 1000.0
        eng = StubEngine(table.clone())
        st = ShardedTable(eng, rank, world, chunks=chunks)
        assert st.chunks == (chunks or 1)
        full = st.build()
        ok_table = (torch.equal(full[:n_news], table * 2 + 1) and eng.hist_table is full
                    and torch.equal(eng.hist_src, table))  # the engine's source table is not modified
        local = torch.arange(rank * 10, rank * 10 + 3 + rank, dtype=torch.float32)
        allsc = gather_scores(local, world)
        want = torch.cat([torch.arange(r * 10, r * 10 + 3 + r, dtype=torch.float32) for r in range(world)])
        q.put((rank, bool(ok_table), bool(torch.equal(allsc, want)), tuple(full.shape)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_news,chunks", [(10, None), (11, None), (11, 2), (23, 3)])
def test_sharded_table_and_gather_gloo(n_news, chunks):
    """chunks > 1: the shard is transformed chunk by chunk, each chunk
    all-gathered asynchronously into the rank-major table (the overlapped path
    RCCL ranks take; ragged chunk sizes and a zero-padded last shard)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_news, q, chunks)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok_table, ok_scores, shape in res:
        assert ok_table and ok_scores
        assert shape == (shard_rows(n_news, world) * world, 1024)


def test_partition_by_cost_balanced_and_contiguous():
    rng = np.random.default_rng(0)
    h = np.clip(rng.geometric(1 / 33, 10000), 1, 600).astype(np.int32)
    c = np.clip(rng.geometric(1 / 37, 10000), 2, 300).astype(np.int32)
    for world in (1, 2, 4, 8):
        b = partition_by_cost(h, c, world, 2048, 2048)
        assert b[0] == 0 and b[-1] == len(h) and np.all(np.diff(b) >= 0) and len(b) == world + 1
        cost = c * (2048 + 8) + h * (2048 + 4)
        parts = np.array([cost[b[i]:b[i + 1]].sum() for i in range(world)])
        assert parts.max() <= cost.sum() / world + cost.max() + 1


def _comm_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from news_recommendation_project_v2_amd.distributed import NrComm
        try:
            NrComm(rank, world)
            q.put((rank, "constructed"))
        except RuntimeError as e:
            q.put((rank, str(e)[:200]))
        # the group is still usable: no rank was left inside a collective
        t = torch.ones(1)
        dist.all_reduce(t)
        q.put((rank, f"after:{int(t.item())}"))
    finally:
        dist.destroy_process_group()


def test_nr_comm_failure_raises_on_every_rank():
    """NrComm's construction is collective.  With no GPU here every
    rank fails (rank 0's id may still be drawn; nr_init cannot run), and every
    rank must raise together and leave the group usable, not hang in a
    broadcast or inside nr_comm_init."""
    from news_recommendation_project_v2_amd import _lib
    if not _lib.LIB_PATH.is_file():
        pytest.skip("libnewsrec_hip.so not built (run __graft_entry__.build())")
    if torch.cuda.is_available():
        pytest.skip("CPU-only check (on a GPU box nr_init succeeds)")
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_comm_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(2 * world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    msgs = {r: [m for rr, m in res if rr == r] for r in range(world)}
    for r in range(world):
        assert msgs[r][0].startswith("NrComm: ") and msgs[r][1] == f"after:{world}", msgs
