"""bf16 GEMMs whose A operand passes the persistent kernel's 32-bit buffer range
(the title encoder's FFN2, [M x 4096] at M > 512 k tokens) run as persistent
launches over row chunks: every row must equal the row of a launch over a
smaller cut of the same rows (bit for bit), and sampled rows the float64 product.
"""
import pytest
import torch


@pytest.mark.gpu
@pytest.mark.parametrize("epilogue", ["resadd", "gelu"])
def test_gemm_rows_past_4gib_of_a_match_smaller_launches(gpu_device, epilogue):
    from news_recommendation_project_v2_amd import ops
    M, K, N = 600_000, 4096, 1024  # A = 4.9 GB > 4 GiB: chunked at 524,288 rows
    g = torch.Generator(device=gpu_device).manual_seed(0)
    a = torch.randn(M, K, device=gpu_device, generator=g, dtype=torch.bfloat16)
    w = (torch.randn(N, K, device=gpu_device, generator=g) * 0.02).to(torch.bfloat16)
    b = torch.randn(N, device=gpu_device, generator=g) * 0.1
    r = torch.randn(M, N, device=gpu_device, generator=g).to(torch.bfloat16) if epilogue == "resadd" else None
    full = ops.gemm(a, w, b, epilogue=epilogue, residual=r)
    cut = 300_000  # both halves fit one persistent launch
    lo = ops.gemm(a[:cut], w, b, epilogue=epilogue, residual=None if r is None else r[:cut])
    hi = ops.gemm(a[cut:], w, b, epilogue=epilogue, residual=None if r is None else r[cut:])
    torch.cuda.synchronize()
    assert torch.equal(full[:cut], lo)
    assert torch.equal(full[cut:], hi)
    rows = torch.tensor([0, 1, 524_287, 524_288, 524_289, M - 1], device=gpu_device)
    ref = a[rows].double() @ w.double().T + b.double()
    if epilogue == "resadd":
        ref = ref + r[rows].double()
    else:
        ref = torch.nn.functional.gelu(ref)
    err = (full[rows].double() - ref).abs().max().item()
    assert err < 0.05 * max(1.0, ref.abs().max().item()), err
