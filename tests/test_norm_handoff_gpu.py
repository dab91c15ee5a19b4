"""Norm hand-offs between GEMMs (csrc/kernels/gemm_8ph.hip epilogue, norm.hip finalizers) vs fp32 PyTorch.

* GroupNorm partials [M / 128, N, 2] written by the v4 wide epilogue (LDS column sums) or by the fallback pass,
  finalised into (scale, shift) -- compared with the standalone statistics kernel and the fp32 reference.
* LayerNorm row moments (mean, rstd) from the epilogue's per-row partials.
* LayerNorm folded into the consuming GEMM: rstd * (x W'^T - mean * s) + b' vs LayerNorm(x) W^T + b in fp32.
* The SD2.1-shaped UNet with the hand-offs on vs off (SHAI_NORM_HANDOFF).
v4 configs: 9 = 256x256, 10 = 256x320, 11 / 12 = their persistent forms; 0 = a v2 tile (fallback passes).
"""
import pytest
import torch

from shai_amd import ops
from shai_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


def rnd(*shape, scale=1.0):
    return (torch.randn(*shape, device="cuda") * scale).to(torch.bfloat16)


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.mark.parametrize("cfg", [9, 10, 11, 12, 0, -1])
@pytest.mark.parametrize("M,N,K", [(4096, 320, 320), (1024, 640, 384), (2048, 1280, 256)])
def test_gemm_gn_partials(cuda, cfg, M, N, K):
    torch.manual_seed(0)
    x, w, b, r = rnd(M, K), rnd(N, K, scale=0.05), rnd(N), rnd(M, N)
    y, part = ops.linear_stats(x, w, b, residual=r, stats="gn", force_cfg=cfg)
    assert rel(y, ref.linear(x, w, b, residual=r)) < 1e-2
    assert part.shape == (M // 128, N, 2)
    assert rel(part, ref.col_partials(y)) < 1e-5


@pytest.mark.parametrize("dc", [0.0, 100.0])
@pytest.mark.parametrize("cfg", [9, 10, 11, 12, 0])
@pytest.mark.parametrize("M,N,K", [(4096, 320, 320), (3000, 640, 320)])
def test_gemm_ln_moments(cuda, cfg, M, N, K, dc):
    """LayerNorm moments of a GEMM output from the v4 epilogue (per-slot shifted (mean, M2), Chan-combined) or the
    fallback pass (sums shifted by the row's first value); dc = a large per-row offset (|mean| / std ~ 100), where
    E[x^2] - mean^2 in fp32 would lose the variance.  Reference: float64 moments of the stored bf16 output."""
    torch.manual_seed(1)
    x, w, b = rnd(M, K), rnd(N, K, scale=0.05), rnd(N)
    r = (torch.randn(M, N, device="cuda") + dc * torch.randn(M, 1, device="cuda").sign()).bfloat16()
    y, mr = ops.linear_stats(x, w, b, residual=r, stats="ln", eps=1e-5, force_cfg=cfg)
    assert mr.shape == (M, 2)
    yd = y.double()
    mean = yd.mean(1)
    rstd = torch.rsqrt(yd.var(1, unbiased=False) + 1e-5)
    assert rel(mr[:, 0], mean) < 1e-5 and rel(mr[:, 1], rstd) < 1e-4


@pytest.mark.parametrize("cfg", [9, 10, 11, 12, -1])
@pytest.mark.parametrize("M,N,K,glu", [(4096, 960, 320, False), (1000, 320, 640, False), (4096, 2560, 320, True)])
def test_folded_layernorm_gemm(cuda, cfg, M, N, K, glu):
    torch.manual_seed(2)
    x = rnd(M, K) + 0.5  # a non-zero row mean
    w, b = rnd(N, K, scale=0.05), rnd(N, scale=0.1)
    gamma, beta = (1.0 + 0.1 * torch.randn(K, device="cuda")).bfloat16(), rnd(K, scale=0.1)
    w2, b2, s = ops.fold_layernorm(w, b, gamma, beta)
    mr = ops.row_moments(x, 1e-5)
    assert rel(mr, ref.row_moments(x, 1e-5)) < 1e-5
    y = ops.linear(x, w2, b2, act="gelu" if glu else None, glu=glu, row_affine=(mr, s), force_cfg=cfg)
    xn = torch.nn.functional.layer_norm(x.float(), (K,), gamma.float(), beta.float(), 1e-5)
    want = ref.linear(xn, w, b, act="gelu" if glu else None, glu=glu)
    assert rel(y, want) < 1.5e-2


@pytest.mark.parametrize("concat", [False, True])
@pytest.mark.parametrize("HW,C", [(4096, 320), (1024, 640), (256, 1280)])
def test_groupnorm_from_partials(cuda, HW, C, concat):
    torch.manual_seed(3)
    N = 4
    x = rnd(N, HW, C) + 0.3
    x2 = rnd(N, HW, C // 2) - 0.2 if concat else None
    gamma, beta = rnd(C + (C // 2 if concat else 0)), rnd(C + (C // 2 if concat else 0))
    p1 = ops.col_partials(x)
    p2 = ops.col_partials(x2) if concat else None
    sc, sh = ops.groupnorm_stats_from_partials(p1, gamma, beta, 32, 1e-5, N, HW, part2=p2)
    sc0, sh0 = ops.groupnorm_stats(x, gamma, beta, 32, 1e-5, x2=x2)
    assert rel(sc, sc0) < 1e-4 and rel(sh, sh0) < 1e-4
    xx = torch.cat([x, x2], -1) if concat else x
    scr, shr = ref.groupnorm_stats(xx, gamma, beta, 32, 1e-5)
    assert rel(sc, scr) < 1e-4 and rel(sh, shr) < 1e-4


@pytest.mark.parametrize("up,temb", [(False, True), (True, False), (False, False)])
def test_conv_gn_partials(cuda, up, temb):
    """3x3 conv (v4 implicit GEMM) with the per-image bias (wide-epilogue bias2d) and residual, writing the
    GroupNorm partials of its output; an 8-channel input (not a v4 conv) takes the fallback pass."""
    torch.manual_seed(4)
    N, H, cin, cout = 4, 16 if up else 32, 320, 320
    x = rnd(N, H, H, cin)
    w = ops.pack_conv_weight(torch.randn(cout, cin, 3, 3, device="cuda").mul(0.02).bfloat16())
    b = rnd(cout)
    t = rnd(N, cout) if temb else None
    OH = 2 * H if up else H
    res = rnd(N, OH, OH, cout)
    y, part = ops.conv2d(x, w, b, 3, 3, 1, 1, upsample=up, temb=t, residual=res, stats="gn")
    want = ref.conv2d(x, w, b, 3, 3, 1, 1, up, None, None, t, res)
    assert rel(y, want) < 1e-2
    assert rel(part, ref.col_partials(y.reshape(-1, cout))) < 1e-5
    x8 = rnd(N, 32, 32, 8)
    w8 = ops.pack_conv_weight(torch.randn(cout, 8, 3, 3, device="cuda").mul(0.1).bfloat16())
    y8, p8 = ops.conv2d(x8, w8, b, 3, 3, 1, 1, stats="gn")
    assert rel(p8, ref.col_partials(y8.reshape(-1, cout))) < 1e-5


@pytest.mark.parametrize("lnout", [True, False])
def test_unet_norm_handoff_matches(cuda, lnout):
    """SD2.1-shaped (reduced-width) UNet: the hand-off forward vs the standalone-norm forward (at the 320-wide level
    either with the LayerNorms computed by the producing out-projections, ops.linear_lnout, or folded into Q / GEGLU)."""
    from shai_amd.models import unet2d
    from shai_amd.models.unet2d import UNet2DConditionModel, UNetConfig
    torch.manual_seed(5)
    cfg = UNetConfig(block_out_channels=(320, 640), layers_per_block=1, attention_heads=(5, 10),
                     cross_attention_dim=256, down_attn=(True, True), time_embed_dim=320)
    m = UNet2DConditionModel(cfg).cuda().eval()
    for p in m.parameters():
        torch.nn.init.normal_(p, std=0.03)
    B, H = 4, 32
    x = torch.randn(B, H, H, 4, device="cuda").bfloat16()
    t = torch.tensor([500.0], device="cuda")
    kv = m.context_kv(torch.randn(B, 77, 256, device="cuda").bfloat16())
    old, old_min, old_lo = unet2d.NORM_HANDOFF, ops.FOLD_MIN_TILES, ops.LNOUT
    try:
        ops.FOLD_MIN_TILES = 0  # fold at this small size too
        ops.LNOUT = lnout
        unet2d.NORM_HANDOFF = True
        y1 = m(x, t, kv)
        unet2d.NORM_HANDOFF = False
        y0 = m(x, t, kv)
    finally:
        unet2d.NORM_HANDOFF, ops.FOLD_MIN_TILES, ops.LNOUT = old, old_min, old_lo
    assert torch.isfinite(y1).all()
    assert rel(y1, y0) < 2e-2


def test_vit_norm_handoff_matches(cuda):
    """ViT-base widths (2 layers, batch 8: 1,576 token rows, not a multiple of 256 -> the producers' moments come
    from the fallback pass, the folded QKV / fc1 GEMMs run on the v4 kernel)."""
    from shai_amd.models import vit
    from shai_amd.models.vit import ViTConfig, ViTEncoderModel
    torch.manual_seed(6)
    c = ViTConfig(num_hidden_layers=2)
    m = ViTEncoderModel(c).cuda().eval()
    for p in m.parameters():
        torch.nn.init.normal_(p, std=0.03)
    px = torch.randn(8, 224, 224, 3, device="cuda").bfloat16()
    old, old_min = vit.NORM_HANDOFF, ops.FOLD_MIN_TILES
    try:
        ops.FOLD_MIN_TILES = 0
        vit.NORM_HANDOFF = True
        y1 = m(px)
        vit.NORM_HANDOFF = False
        y0 = m(px)
    finally:
        vit.NORM_HANDOFF, ops.FOLD_MIN_TILES = old, old_min
    assert torch.isfinite(y1).all()
    assert rel(y1, y0) < 2e-2
