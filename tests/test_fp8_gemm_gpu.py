"""W8A8 fp8 MFMA GEMM (gemm_f8.hip) and the per-row activation quantiser vs fp32 torch references."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from shai_amd import ops  # noqa: E402
from shai_amd.ops import reference as ref  # noqa: E402


@pytest.fixture(scope="module")
def cuda():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda")


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("M,K", [(1, 64), (300, 4096), (17, 28672)])
@pytest.mark.parametrize("rms", [False, True])
def test_quant_rows_fp8_matches_reference(cuda, M, K, rms):
    torch.manual_seed(M + K)
    x = (torch.randn(M, K, device=cuda) * 3).bfloat16()
    x[0, 5] = 40.0                                  # an outlier sets row 0's scale
    a8, s = ops.quant_rows_fp8(x, 1e-5 if rms else None)
    r8, rs = ref.quant_rows_fp8(x, 1e-5 if rms else None)
    torch.testing.assert_close(s, rs, rtol=1e-5, atol=0)
    # same e4m3 codes up to one ulp of round-to-nearest ties
    diff = (a8.float() - r8.float()).abs() / r8.float().abs().clamp(min=2 ** -6)
    assert (diff > 0.13).sum().item() == 0
    if not rms:
        assert _rel(a8.float() * s[:, None], x) < 0.04


@pytest.mark.parametrize("M,N,K", [(256, 512, 512), (300, 1000, 4096), (4096, 4096, 4096), (129, 128, 208)])
@pytest.mark.parametrize("cfg", [0, 1, 2])
def test_gemm_f8_matches_dequantized_fp32(cuda, M, N, K, cfg):
    """Exact fp8 operands (quantised once), fp32 product of the same codes: only accumulation order differs."""
    torch.manual_seed(M * 3 + N + K)
    x = torch.randn(M, K, device=cuda).bfloat16()
    w = (torch.randn(N, K, device=cuda) / K ** 0.5).bfloat16()
    a8, a_s = ops.quant_rows_fp8(x)
    w8, w_s = ops.quantize_fp8_rows(w)
    b = torch.randn(N, device=cuda).bfloat16()
    y = ops.gemm_f8(a8, w8, a_s, w_s, bias=b, cfg=cfg)
    want = ref.gemm_f8(a8, w8, a_s, w_s, bias=b)
    assert _rel(y, want) < 5e-3
    assert _rel(y, ref.linear(x, w, b)) < 6e-2     # vs the bf16 product: fp8 rounding of both operands


def test_gemm_f8_epilogues_glu_residual(cuda):
    torch.manual_seed(3)
    M, N, K = 520, 1024, 1024
    x = torch.randn(M, K, device=cuda).bfloat16()
    w = (torch.randn(N, K, device=cuda) / K ** 0.5).bfloat16()
    a8, a_s = ops.quant_rows_fp8(x)
    w8, w_s = ops.quantize_fp8_rows(w)
    y = ops.gemm_f8(a8, w8, a_s, w_s, act="silu", glu=True)
    assert _rel(y, ref.gemm_f8(a8, w8, a_s, w_s, act="silu", glu=True)) < 5e-3
    r = torch.randn(M, N, device=cuda).bfloat16()
    y2 = ops.gemm_f8(a8, w8, a_s, w_s, residual=r, res_alpha=0.5)
    assert _rel(y2, ref.gemm_f8(a8, w8, a_s, w_s, residual=r, res_alpha=0.5)) < 5e-3


def test_linear_fp8_prefill_w8a8_with_folded_rmsnorm(cuda):
    """ops.linear with fp8 weights on a prefill-sized problem takes the W8A8 path; the RMSNorm rstd rides in the
    activation row scale."""
    torch.manual_seed(4)
    M, N, K = 384, 2048, 4096
    x = (torch.randn(M, K, device=cuda) * 2).bfloat16()
    w = (torch.randn(N, K, device=cuda) / K ** 0.5).bfloat16()
    w8, w_s = ops.quantize_fp8_rows(w)
    y = ops.linear(x, w8, rms_eps=1e-5, w_scale=w_s)
    xn = ref.rmsnorm(x, None, 1e-5)[0]
    assert _rel(y, ref.linear(xn, w)) < 6e-2
