"""Host <-> device legs of the drop-in API through the library's pinned staging
ring (include/newsrec.h nr_copy_h2d / nr_copy_d2h, csrc/xfer.hip; VERDICT r5
#6).  Byte-exact round trips at every size class the pipeline has: empty, one
byte, the single-bounce limit (1 MiB) and one past it, a ragged multi-chunk
size that is not a multiple of the thread slices, and MIND-large-dev index
sizes; stream order both ways (a device write queued before d2h is seen, an
h2d is complete before a kernel queued after it reads it); and the engine /
API paths that now use it return the same scores as before."""
import numpy as np
import pytest
import torch

from news_recommendation_project_v2_amd import _lib, ops


@pytest.mark.gpu
@pytest.mark.parametrize("nbytes", [0, 1, 4095, (1 << 20), (1 << 20) + 1, 4 * (8 << 20) + 12345,
                                    9 * (8 << 20) + 7, 111_000_001])
def test_round_trip_bytes(gpu_device, nbytes):
    rng = np.random.default_rng(nbytes)
    src = rng.integers(0, 256, nbytes, dtype=np.uint8)
    d = torch.empty(nbytes, dtype=torch.uint8, device=gpu_device)
    ops.h2d(d, src)
    torch.cuda.synchronize()
    assert torch.equal(d.cpu(), torch.from_numpy(src))  # read back through torch, independent of d2h
    back = np.full(nbytes, 7, dtype=np.uint8)
    ops.d2h(back, d)
    np.testing.assert_array_equal(back, src)


@pytest.mark.gpu
def test_stream_order(gpu_device):
    """d2h after a kernel queued on the same stream sees its result; a kernel
    queued after h2d reads the uploaded bytes (no explicit sync in between)."""
    n = 3 * (8 << 20) // 4 + 999
    x = torch.zeros(n, dtype=torch.float32, device=gpu_device)
    host = np.arange(n, dtype=np.float32)
    ops.h2d(x, host)
    y = x * 2 + 1  # queued after the copies
    out = np.empty(n, dtype=np.float32)
    ops.d2h(out, y)
    np.testing.assert_array_equal(out, host * 2 + 1)
    # CPU tensors on the host side, int64
    t = torch.arange(5_000_003, dtype=torch.int64)
    d = ops.to_device(t, gpu_device)
    assert d.dtype == torch.int64 and torch.equal(d.cpu(), t)
    h = ops.to_host(d + 1)
    np.testing.assert_array_equal(h, t.numpy() + 1)


@pytest.mark.gpu
def test_copy_errors(gpu_device):
    d = torch.empty(16, dtype=torch.uint8, device=gpu_device)
    with pytest.raises(_lib.NewsRecHIPError):
        ops.h2d(d, np.zeros(8, dtype=np.uint8))  # byte count mismatch
    with pytest.raises(_lib.NewsRecHIPError):
        ops.d2h(np.zeros(16, dtype=np.uint8)[::2].copy()[:4], d)
    lib = _lib.load()
    buf = np.zeros(16, dtype=np.uint8)
    assert lib.nr_copy_h2d(buf.ctypes.data, buf.ctypes.data, 16, None) == -1  # host dst refused
    assert "nr_copy_h2d" in lib.nr_last_error().decode()
    assert lib.nr_copy_d2h(buf.ctypes.data, None, 16, None) == -1
    assert lib.nr_copy_h2d(d.data_ptr(), buf.ctypes.data, -1, None) == -1
    assert lib.nr_copy_h2d(d.data_ptr(), buf.ctypes.data, 0, None) == 0


@pytest.mark.gpu
def test_api_scores_unchanged_by_staging(gpu_device):
    """get_final_second_attention_score with the staged legs against the same
    engine fed and read through torch's own copies: identical scores and ranks."""
    from news_recommendation_project_v2_amd import data_model_helper as dmh
    from news_recommendation_project_v2_amd import synthetic
    from news_recommendation_project_v2_amd import weights as W
    from news_recommendation_project_v2_amd.engine import PoolScoreEngine
    from news_recommendation_project_v2_amd.latent_attention import LatentAttentionModel
    m = LatentAttentionModel()
    m.load_state_dict(W.latent_attention_state_dict(5))
    m = m.to(gpu_device).eval()
    im = synthetic.mind_impressions(3000, 2000, seed=5)
    table = torch.randn(3000, 1024, generator=torch.Generator().manual_seed(5))
    hb = np.ones(im.n_imp, dtype=bool)
    dmh.PROFILE = True
    try:
        got = dmh.get_final_second_attention_score(im.hist_idx, im.hist_len, im.cand_idx, im.cand_len, table, hb, m,
                                                   dtype=torch.bfloat16)
        t = dict(dmh.LAST_TIMINGS)
    finally:
        dmh.PROFILE = False
    assert set(t) == {"setup_upload", "device", "download", "host", "total"}, t
    eng = PoolScoreEngine(m, dtype=torch.bfloat16, device=gpu_device)
    eng.cand_table = table.to(gpu_device).to(torch.bfloat16)
    eng.hist_src = eng.cand_table
    eng.load_impressions(im.hist_idx, im.hist_len, im.cand_idx, im.cand_len)
    s, _ = eng.step()
    np.testing.assert_array_equal(got["scores"], s.cpu().numpy())
    r = eng.rank(s).cpu().numpy()
    np.testing.assert_array_equal(np.concatenate(list(got["grouped_scores"])), r)
