"""The persistent bf16 GEMM's half-tile tail (gemm.hip gemm256t_kernel units;
include/newsrec.h nr_set_gemm_half_tail): when the output tiles leave a last
partial round of at most half the grid, those tiles run as 128-row halves on
wave group 0 alone.  Every element keeps its K chain and epilogue, so the
output must be bit-identical with the tail on and off, for every epilogue the
persistent kernel serves, at shapes where the split triggers (M = 72,023:
1,128 tiles at N = 1024 leave 104 = 208 halves; N = 512: 52; M = 8,320, N = 512:
66 tiles, all halves) and where it does not (N = 4096: 160 > 128)."""
import pytest
import torch


def _run(ops, on, **kw):
    ops.set_gemm_half_tail(on)
    try:
        out = ops.gemm(**kw)
        torch.cuda.synchronize()
        return out
    finally:
        ops.set_gemm_half_tail(True)


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K,epilogue", [
    (72_023, 1024, 512, "resadd"), (72_023, 1024, 4096, "resadd"), (72_023, 512, 1024, "softmax64"),
    (72_023, 8192, 1024, "geglu"), (72_023, 4096, 1024, "relu"), (72_023, 1024, 4096, "exp"),
    (8_320, 512, 1024, "none"), (8_320, 1024, 256, "gelu"), (300, 1024, 512, "resadd"),
])
def test_half_tail_is_bit_identical(gpu_device, M, N, K, epilogue):
    from news_recommendation_project_v2_amd import ops
    g = torch.Generator(device=gpu_device).manual_seed(M + N + K)
    a = torch.randn(M, K, device=gpu_device, generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, device=gpu_device, generator=g) * K ** -0.5).to(torch.bfloat16)
    b = torch.randn(N, device=gpu_device, generator=g) * 0.1
    r = torch.randn(M, N, device=gpu_device, generator=g).to(torch.bfloat16) if epilogue == "resadd" else None
    kw = dict(a=a, w=w, bias=b, epilogue=epilogue, residual=r)
    on, off = _run(ops, True, **kw), _run(ops, False, **kw)
    assert torch.equal(on, off)
    rows = torch.tensor([0, 127, 128, 255, M // 2, M - 129, M - 128, M - 1], device=gpu_device).clamp(max=M - 1)
    ref = a[rows].double() @ w.double().T + b.double()
    if epilogue == "resadd":
        ref = ref + r[rows].double()
    elif epilogue == "relu":
        ref = ref.clamp(min=0)
    elif epilogue == "exp":
        ref = ref.exp()
    elif epilogue == "gelu":
        ref = torch.nn.functional.gelu(ref)
    elif epilogue == "geglu":
        blk = ref.view(len(rows), -1, 2, 32)  # W rows interleaved in 32-row (a, g) blocks
        ref = (blk[:, :, 0] * torch.nn.functional.gelu(blk[:, :, 1])).reshape(len(rows), -1)
    elif epilogue == "softmax64":
        ref = torch.softmax(ref.view(len(rows), -1, 64), -1).view(len(rows), -1)
    err = (on[rows].double() - ref).abs().max().item()
    assert err < 0.02 * max(1.0, ref.abs().max().item()), err


@pytest.mark.gpu
@pytest.mark.parametrize("pooler", ["latent", "final"])
def test_half_tail_transform_table_identical(gpu_device, pooler):
    """The whole per-news transform (LN-folded S, B, GEGLU ff1, ff2 / the
    FinalAttention chain) with the tail on and off: the same table bit for bit."""
    from news_recommendation_project_v2_amd import ops
    from news_recommendation_project_v2_amd import weights as W
    from news_recommendation_project_v2_amd.engine import PoolScoreEngine
    from news_recommendation_project_v2_amd.latent_attention import LatentAttentionModel
    from news_recommendation_project_v2_amd.modeling_utils import FinalAttention
    m = LatentAttentionModel() if pooler == "latent" else FinalAttention(1024, 4096)
    m.load_state_dict(W.latent_attention_state_dict(5) if pooler == "latent" else W.final_attention_state_dict(5))
    table = W.news_table(5, 72_023, 1024, name="half_tail")
    eng = PoolScoreEngine(m.to(gpu_device).eval(), dtype=torch.bfloat16, device=gpu_device).load_news(table)
    on = eng.transform().clone()
    ops.set_gemm_half_tail(False)
    try:
        off = eng.transform().clone()
    finally:
        ops.set_gemm_half_tail(True)
    torch.cuda.synchronize()
    assert torch.equal(on, off)
