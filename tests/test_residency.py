"""C-ABI error contract for caller mistakes:
a host (CPU-tensor) pointer handed to an entry returns NR_ERR_INVALID with a
message naming the argument, instead of reaching an async kernel that faults
the GPU (the round-2 fault of gpurun_out/enc2.log: a CPU-resident model's
weights passed to nr_encoder_forward).  After the refused call the device and
torch's error state are clean, and the same call with device tensors runs."""
import ctypes

import numpy as np
import pytest
import torch

from news_recommendation_project_v2_amd import _lib


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr())


@pytest.mark.gpu
def test_pool_score_refuses_cpu_tensors(gpu_device):
    lib = _lib.load()
    n_news, dev = 64, gpu_device
    tab_h = torch.randn(n_news, 1024)
    off_h = torch.tensor([0, 3, 5], dtype=torch.int64)
    idx_h = torch.tensor([1, 2, 3, 4, 5], dtype=torch.int32)
    tab, off, idx = tab_h.to(dev), off_h.to(dev), idx_h.to(dev)
    inv = torch.ones(n_news, device=dev)
    scores = torch.empty(5, device=dev)
    cases = {"hist_table": (tab_h, off, idx), "hist_off": (tab, off_h, idx), "cand_idx": (tab, off, idx_h)}
    for name, (t, o, i) in cases.items():
        rc = lib.nr_pool_score(_lib.NR_POOL_LATENT, _lib.NR_F32, 1024, _ptr(t), 1024, _ptr(tab), 1024, _ptr(inv),
                               _ptr(idx), _ptr(o), _ptr(i), _ptr(off), 2, _ptr(scores), None, None)
        msg = lib.nr_last_error().decode()
        assert rc == -1, msg  # NR_ERR_INVALID
        assert f"`{name}`" in msg and "not device memory" in msg, msg
    torch.cuda.synchronize()
    # no stale HIP error is left for torch's own launch checks; the device call runs
    (tab * 2).sum().item()
    rc = lib.nr_pool_score(_lib.NR_POOL_LATENT, _lib.NR_F32, 1024, _ptr(tab), 1024, _ptr(tab), 1024, _ptr(inv),
                           _ptr(idx), _ptr(off), _ptr(idx), _ptr(off), 2, _ptr(scores), None,
                           ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0, lib.nr_last_error()
    torch.cuda.synchronize()
    assert torch.isfinite(scores).all()


@pytest.mark.gpu
def test_encoder_forward_refuses_host_weights(gpu_device):
    """The enc2.log case itself: layer weights of a CPU-resident model."""
    lib = _lib.load()
    dev = gpu_device
    D, F, V, P = 1024, 4096, 100, 514

    def w(*shape, on=dev):
        return (torch.randn(*shape) * 0.02).to(on)

    layer_cpu = dict(wqkv=w(3 * D, D, on="cpu"), bqkv=w(3 * D), wo=w(D, D), bo=w(D), ln1_g=torch.ones(D, device=dev),
                     ln1_b=torch.zeros(D, device=dev), w1=w(F, D), b1=w(F), w2=w(D, F), b2=w(D),
                     ln2_g=torch.ones(D, device=dev), ln2_b=torch.zeros(D, device=dev))
    layers = (_lib.EncoderLayer * 1)()
    for k, v in layer_cpu.items():
        setattr(layers[0], k, v.data_ptr())
    word, pos, typ = w(V, D), w(P, D), w(1, D)
    g, b = torch.ones(D, device=dev), torch.zeros(D, device=dev)
    lens = torch.tensor([5, 7], dtype=torch.int32, device=dev)
    ids = torch.randint(3, V, (12,), dtype=torch.int32, device=dev)
    pooled = torch.empty(2, D, device=dev)
    nbytes = lib.nr_encoder_workspace_bytes(_lib.NR_F32, 12, 2)
    ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    def run():
        return lib.nr_encoder_forward(_lib.NR_F32, 1, layers, _ptr(word), V, _ptr(pos), P, _ptr(typ), _ptr(g),
                                      _ptr(b), 1e-5, 2, 12, _ptr(lens), _ptr(ids), _lib.NR_POOL_MEAN, _ptr(pooled),
                                      None, None, _ptr(ws), nbytes, stream)

    rc = run()
    msg = lib.nr_last_error().decode()
    assert rc == -1 and "`L.wqkv`" in msg and "not device memory" in msg, msg
    # host ids (the offsets/ids path) are refused too
    ids_h = ids.cpu()
    rc = lib.nr_encoder_forward(_lib.NR_F32, 0, None, _ptr(word), V, _ptr(pos), P, _ptr(typ), _ptr(g), _ptr(b), 1e-5,
                                2, 12, _ptr(lens), _ptr(ids_h), _lib.NR_POOL_MEAN, _ptr(pooled), None, None, _ptr(ws),
                                nbytes, stream)
    assert rc == -1 and "`ids`" in lib.nr_last_error().decode()
    # the same call with the weights moved to the device runs and pools finite rows
    layer_cpu["wqkv"] = layer_cpu["wqkv"].to(dev)
    layers[0].wqkv = layer_cpu["wqkv"].data_ptr()
    assert run() == 0, lib.nr_last_error()
    torch.cuda.synchronize()
    assert torch.isfinite(pooled).all()
    np.testing.assert_array_less(0.0, pooled.abs().sum(1).cpu().numpy())


@pytest.mark.gpu
def test_residency_flush_drops_freed_ranges(gpu_device):
    """verified ranges are cached per thread; after torch returns a
    segment to the driver (empty_cache) its address range is no longer device
    memory.  nr_residency_flush (called by _lib.empty_cache) drops the cached
    ranges, so the freed address is verified again and refused.  Only the
    query entry is called with the stale pointer: nothing is launched on it."""
    lib = _lib.load()
    t = torch.empty(512 << 20, dtype=torch.uint8, device=gpu_device)  # its own 512 MiB segment
    p = ctypes.c_void_p(t.data_ptr() + (256 << 20))
    assert lib.nr_is_device_pointer(p) == 1
    del t
    torch.cuda.synchronize()
    torch.cuda.empty_cache()  # the segment goes back to the driver; the range is still cached
    assert lib.nr_is_device_pointer(p) == 1  # the stale verdict the flush exists for
    # the HIP runtime may keep a freed range mapped (its own pool; seen in the
    # full suite): the flush must then give the driver's current verdict
    hip = ctypes.CDLL("libamdhip64.so")
    attr = (ctypes.c_ubyte * 128)()
    driver_says_device = hip.hipPointerGetAttributes(attr, p) == 0 and int.from_bytes(bytes(attr[:4]), "little") in (2, 3)
    hip.hipGetLastError()  # a refused query leaves the runtime's last error set
    _lib.empty_cache()  # empty_cache + nr_residency_flush
    assert lib.nr_is_device_pointer(p) == int(driver_says_device)
    (torch.ones(4, device=gpu_device) * 2).sum().item()  # no HIP error left behind
    assert lib.nr_is_device_pointer(ctypes.c_void_p(torch.ones(4, device=gpu_device).data_ptr())) == 1
