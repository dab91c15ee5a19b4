"""fp8 (OCP e4m3) CPU references: per-row activation quantisation and the W8A8 product that the gfx950
kernels (gemm_f8.hip) are checked against, plus the fp8-weight ops.linear fallback on CPU."""
import torch

from shai_amd import ops
from shai_amd.ops import reference as ref


def test_quant_rows_fp8_reference_roundtrip_and_rms_scale():
    torch.manual_seed(0)
    x = (torch.randn(5, 256) * 4).bfloat16()
    a8, s = ref.quant_rows_fp8(x)
    assert a8.dtype == torch.float8_e4m3fn and s.shape == (5,)
    assert a8.float().abs().amax(-1).allclose(torch.full((5,), 448.0))       # the row max maps to e4m3 max
    rel = ((a8.float() * s[:, None] - x.float()).norm() / x.float().norm()).item()
    assert rel < 0.04
    _, s_rms = ref.quant_rows_fp8(x, 1e-5)
    rstd = torch.rsqrt(x.float().pow(2).mean(-1) + 1e-5)
    torch.testing.assert_close(s_rms, s * rstd)


def test_gemm_f8_reference_matches_bf16_product():
    torch.manual_seed(1)
    x = torch.randn(33, 512).bfloat16()
    w = (torch.randn(96, 512) / 512 ** 0.5).bfloat16()
    b = torch.randn(96).bfloat16()
    a8, a_s = ref.quant_rows_fp8(x)
    w8, w_s = ops.quantize_fp8_rows(w)
    y = ref.gemm_f8(a8, w8, a_s, w_s, bias=b)
    want = ref.linear(x, w, b)
    assert ((y.float() - want.float()).norm() / want.float().norm()).item() < 0.06
    g = ref.gemm_f8(a8, w8, a_s, w_s, act="silu", glu=True)
    assert g.shape == (33, 48)


def test_linear_fp8_weights_cpu_fallback_dequantizes():
    torch.manual_seed(2)
    x = torch.randn(80, 256).bfloat16()
    w = (torch.randn(64, 256) / 16).bfloat16()
    w8, w_s = ops.quantize_fp8_rows(w)
    y = ops.linear(x, w8, w_scale=w_s)
    want = ref.linear(x, ops.dequant_fp8(w8, w_s))
    torch.testing.assert_close(y, want)
