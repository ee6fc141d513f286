"""The library's own RCCL communicator (include/newsrec.h nr_comm_* /
nr_allgather; SURVEY §8(b) "nr_allgather (RCCL communicator handle created from
a unique id passed by the host)", §8(e) phase B).  RCCL needs one GPU per rank,
so on the one-GPU box the collective runs on a one-rank communicator: the
gathered table must equal torch.distributed's all_gather_into_tensor on a
one-rank RCCL group and the one-shot transform bit for bit.  The multi-rank
run is the driver's 8-GPU bench (bench.py reports `nr_allgather` beside
torch's all-gather there, bit-identity checked on every rank)."""
import ctypes

import pytest
import torch

from news_recommendation_project_v2_amd import _lib
from news_recommendation_project_v2_amd import weights as W


@pytest.fixture(scope="module")
def lib():
    if not _lib.LIB_PATH.is_file():
        pytest.skip("libnewsrec_hip.so not built (run __graft_entry__.build())")
    return _lib.load()


def test_comm_argument_errors(lib):
    """Caller mistakes are refused before RCCL is touched (no device needed)."""
    h = ctypes.c_void_p()
    idb = (ctypes.c_ubyte * 128)()
    assert lib.nr_comm_init(ctypes.byref(h), idb, 2, 2) == -1  # rank out of range
    assert "rank 2 of 2" in lib.nr_last_error().decode()
    assert lib.nr_comm_init(None, idb, 1, 0) == -1
    assert lib.nr_comm_init_timeout(ctypes.byref(h), idb, 1, 1, 1000) == -1
    assert lib.nr_comm_init_timeout(None, idb, 1, 0, 1000) == -1
    assert lib.nr_allgather(None, None, None, 16, None) == -1
    assert lib.nr_comm_destroy(None) == 0
    assert lib.nr_rccl_version() >= 0


@pytest.mark.gpu
@pytest.mark.parametrize("pooler", ["latent", "final"])
def test_nr_allgather_one_rank_matches_torch(gpu_device, pooler, tmp_path):
    import torch.distributed as dist
    from news_recommendation_project_v2_amd.distributed import NrComm, ShardedTable
    from news_recommendation_project_v2_amd.engine import PoolScoreEngine
    from news_recommendation_project_v2_amd.latent_attention import LatentAttentionModel
    from news_recommendation_project_v2_amd.modeling_utils import FinalAttention
    lib = _lib.load()
    assert lib.nr_rccl_version() > 0
    dist.init_process_group("nccl", init_method=f"file://{tmp_path / 'store'}", rank=0, world_size=1,
                            device_id=gpu_device)
    comm = None
    try:
        m = LatentAttentionModel() if pooler == "latent" else FinalAttention(1024, 4096)
        m.load_state_dict(W.latent_attention_state_dict(9) if pooler == "latent" else W.final_attention_state_dict(9))
        table = W.news_table(9, 5003, 1024, name="comm")
        eng = PoolScoreEngine(m.to(gpu_device).eval(), dtype=torch.bfloat16, device=gpu_device).load_news(table)
        want = eng.transform().clone()
        via_torch = ShardedTable(eng, 0, 1).build().clone()
        comm = NrComm(0, 1)
        via_nr = ShardedTable(eng, 0, 1, comm=comm).build()
        torch.cuda.synchronize()
        assert torch.equal(via_nr, via_torch)
        assert torch.equal(via_nr[:5003], want)
        # out of place, odd byte count: recv = send
        src = torch.randint(0, 255, (12345,), dtype=torch.uint8, device=gpu_device)
        dst = torch.zeros_like(src)
        comm.allgather(src, dst)
        ref = torch.zeros_like(src)
        dist.all_gather_into_tensor(ref, src)
        torch.cuda.synchronize()
        assert torch.equal(dst, src) and torch.equal(dst, ref)
    finally:
        if comm is not None:
            comm.close()
        dist.destroy_process_group()


@pytest.mark.gpu
def test_comm_init_timeout_when_a_peer_never_joins(gpu_device):
    """nr_comm_init_timeout for rank 0 of a 2-rank communicator whose rank 1 never
    calls in: the non-blocking init is aborted at the deadline and the call
    returns NR_ERR_TIMEOUT (-4) naming the rank, instead of blocking forever
    (a stuck rank must fail with a record).  A second, one-rank
    communicator formed afterwards still works (the abort left RCCL usable)."""
    import time
    lib = _lib.load()
    _lib.check(lib.nr_init(gpu_device.index or 0), "nr_init")
    idb = (ctypes.c_ubyte * 128)()
    _lib.check(lib.nr_comm_unique_id(ctypes.cast(idb, ctypes.POINTER(ctypes.c_ubyte))), "nr_comm_unique_id")
    h = ctypes.c_void_p()
    t0 = time.perf_counter()
    rc = lib.nr_comm_init_timeout(ctypes.byref(h), idb, 2, 0, 2000)
    dt = time.perf_counter() - t0
    msg = lib.nr_last_error().decode()
    print(f"rc {rc} after {dt:.2f}s: {msg}")
    assert rc == -4 and "did not form within 2000 ms" in msg and "rank 0 of 2" in msg, (rc, msg)
    assert 1.9 <= dt <= 30.0, dt
    assert not h.value
    idb1 = (ctypes.c_ubyte * 128)()
    _lib.check(lib.nr_comm_unique_id(ctypes.cast(idb1, ctypes.POINTER(ctypes.c_ubyte))), "nr_comm_unique_id")
    h1 = ctypes.c_void_p()
    _lib.check(lib.nr_comm_init_timeout(ctypes.byref(h1), idb1, 1, 0, 30000), "nr_comm_init_timeout")
    x = torch.arange(1024, dtype=torch.uint8, device=gpu_device)
    y = torch.zeros_like(x)
    _lib.check(lib.nr_allgather(h1, x.data_ptr(), y.data_ptr(), 1024, torch.cuda.current_stream().cuda_stream),
               "nr_allgather")
    torch.cuda.synchronize()
    assert torch.equal(x, y)
    _lib.check(lib.nr_comm_destroy(h1), "nr_comm_destroy")
