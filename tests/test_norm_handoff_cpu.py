"""CPU reference paths of the norm hand-offs (the GPU kernels are checked against the same functions in
test_norm_handoff_gpu.py): LayerNorm folding algebra, GroupNorm from partials (with concat), and the UNet forward
with hand-offs on vs off."""
import torch

from shai_amd import ops
from shai_amd.ops import reference as ref


def rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def test_fold_layernorm_matches_layernorm_then_linear():
    torch.manual_seed(0)
    M, K, N = 64, 96, 40
    x = (torch.randn(M, K) + 0.7).bfloat16()
    w, b = (torch.randn(N, K) * 0.1).bfloat16(), (torch.randn(N) * 0.1).bfloat16()
    gamma, beta = (1 + 0.1 * torch.randn(K)).bfloat16(), (0.1 * torch.randn(K)).bfloat16()
    w2, b2, s = ops.fold_layernorm(w, b, gamma, beta)
    mr = ops.row_moments(x, 1e-5)
    y = ops.linear(x, w2, b2, row_affine=(mr, s))
    xn = torch.nn.functional.layer_norm(x.float(), (K,), gamma.float(), beta.float(), 1e-5)
    assert rel(y, ref.linear(xn, w, b)) < 1e-2
    y_st, mr2 = ops.linear_stats(x, w, b, stats="ln", eps=1e-6)
    assert rel(mr2, ref.row_moments(y_st, 1e-6)) < 1e-6


def test_groupnorm_from_partials_concat():
    torch.manual_seed(1)
    N, HW, C1, C2 = 3, 256, 64, 32
    x, x2 = torch.randn(N, HW, C1).bfloat16(), (torch.randn(N, HW, C2) + 1).bfloat16()
    gamma, beta = torch.randn(C1 + C2).bfloat16(), torch.randn(C1 + C2).bfloat16()
    sc, sh = ops.groupnorm_stats_from_partials(ops.col_partials(x), gamma, beta, 8, 1e-5, N, HW,
                                               part2=ops.col_partials(x2))
    sc0, sh0 = ref.groupnorm_stats(torch.cat([x, x2], -1), gamma, beta, 8, 1e-5)
    assert rel(sc, sc0) < 1e-5 and rel(sh, sh0) < 1e-5


def test_conv_stats_shapes():
    torch.manual_seed(2)
    x = torch.randn(2, 16, 16, 8).bfloat16()
    w = ops.pack_conv_weight((torch.randn(16, 8, 3, 3) * 0.1).bfloat16())
    y, p = ops.conv2d(x, w, None, 3, 3, 1, 1, stats="gn")
    assert p.shape == (4, 16, 2) and rel(p, ref.col_partials(y.reshape(-1, 16))) < 1e-6
    y, p = ops.conv2d(torch.randn(2, 8, 8, 8).bfloat16(), w, None, 3, 3, 1, 1, stats="gn")
    assert p is None  # 64-pixel images: a 128-row block would straddle two images


def test_unet_norm_handoff_cpu():
    from shai_amd.models import unet2d
    from shai_amd.models.unet2d import UNet2DConditionModel, UNetConfig
    torch.manual_seed(3)
    cfg = UNetConfig.tiny()
    m = UNet2DConditionModel(cfg).eval()
    for p in m.parameters():
        torch.nn.init.normal_(p, std=0.05)
    x = torch.randn(2, 16, 16, 4).bfloat16()
    t = torch.tensor([500.0])
    kv = m.context_kv(torch.randn(2, 77, cfg.cross_attention_dim).bfloat16())
    old, old_min = unet2d.NORM_HANDOFF, ops.FOLD_MIN_TILES
    try:
        ops.FOLD_MIN_TILES = 0  # fold at this small size too
        unet2d.NORM_HANDOFF = True
        y1 = m(x, t, kv)
        unet2d.NORM_HANDOFF = False
        y0 = m(x, t, kv)
    finally:
        unet2d.NORM_HANDOFF, ops.FOLD_MIN_TILES = old, old_min
    assert rel(y1, y0) < 1e-2


def test_unet_merged_proj_out_cpu():
    """The last transformer block's FF down projection merged into proj_out (one GEMM over [GEGLU out | residual
    stream] with [W_po W_fo | W_po]) matches the two GEMMs, and the merged weights follow a weight update."""
    from shai_amd.models import unet2d
    from shai_amd.models.unet2d import UNet2DConditionModel, UNetConfig
    torch.manual_seed(4)
    cfg = UNetConfig.tiny()
    m = UNet2DConditionModel(cfg).eval()
    for p in m.parameters():
        torch.nn.init.normal_(p, std=0.05)
    x = torch.randn(2, 16, 16, 4).bfloat16()
    t = torch.tensor([500.0])
    kv = m.context_kv(torch.randn(2, 77, cfg.cross_attention_dim).bfloat16())
    old, old_min, old_h = unet2d.MERGE_PROJ_OUT, ops.FOLD_MIN_TILES, unet2d.NORM_HANDOFF
    try:
        ops.FOLD_MIN_TILES = 0  # the folded (forward_parts) path at this small size too
        unet2d.NORM_HANDOFF = True
        unet2d.MERGE_PROJ_OUT = True
        y1 = m(x, t, kv)
        assert any(getattr(mod, "_po_merged", None) is not None for mod in m.modules()), "merged path not taken"
        unet2d.MERGE_PROJ_OUT = False
        y0 = m(x, t, kv)
        assert rel(y1, y0) < 1e-2
        tr = next(mod for mod in m.modules() if isinstance(mod, unet2d.Transformer2DModel))
        with torch.no_grad():
            tr.proj_out.weight.mul_(-1.5)
        unet2d.MERGE_PROJ_OUT = True
        y1 = m(x, t, kv)
        unet2d.MERGE_PROJ_OUT = False
        y0 = m(x, t, kv)
        assert rel(y1, y0) < 1e-2
    finally:
        unet2d.MERGE_PROJ_OUT, ops.FOLD_MIN_TILES, unet2d.NORM_HANDOFF = old, old_min, old_h


def test_unet_proj_in_groupnorm_fold_cpu():
    """Transformer2D input GroupNorm folded into proj_in per image (per-image weight slices + per-image bias, no
    normalised activation) matches GroupNorm apply + proj_in; ops.linear_wslices matches its definition."""
    from shai_amd.models import unet2d
    from shai_amd.models.unet2d import UNet2DConditionModel, UNetConfig
    torch.manual_seed(5)
    x, w, b2 = torch.randn(512, 32).bfloat16(), torch.randn(2, 48, 32).bfloat16(), torch.randn(2, 48).bfloat16()
    y, st = ops.linear_wslices(x, w, b2, 256, stats="ln", eps=1e-5)
    want = torch.cat([x[:256].float() @ w[0].float().t() + b2[0].float(), x[256:].float() @ w[1].float().t() + b2[1].float()])
    assert rel(y, want) < 1e-2 and st.shape == (512, 2)
    cfg = UNetConfig.tiny()
    m = UNet2DConditionModel(cfg).eval()
    for p in m.parameters():
        torch.nn.init.normal_(p, std=0.05)
    xs = torch.randn(2, 16, 16, 4).bfloat16()
    t = torch.tensor([500.0])
    kv = m.context_kv(torch.randn(2, 77, cfg.cross_attention_dim).bfloat16())
    tr = next(mod for mod in m.modules() if isinstance(mod, unet2d.Transformer2DModel))
    old, old_min, old_h = unet2d.GN_FOLD_PROJ_IN, ops.FOLD_MIN_TILES, unet2d.NORM_HANDOFF
    try:
        ops.FOLD_MIN_TILES = 0
        unet2d.NORM_HANDOFF = True
        unet2d.GN_FOLD_PROJ_IN = True
        assert tr._gn_fold_ok(torch.empty(2, 16, 16, tr.proj_in.cin_p)), "fold not eligible at the tiny config"
        y1 = m(xs, t, kv)
        unet2d.GN_FOLD_PROJ_IN = False
        y0 = m(xs, t, kv)
    finally:
        unet2d.GN_FOLD_PROJ_IN, ops.FOLD_MIN_TILES, unet2d.NORM_HANDOFF = old, old_min, old_h
    assert rel(y1, y0) < 1e-2


def test_vit_norm_handoff_cpu():
    from shai_amd.models import vit
    from shai_amd.models.vit import ViTConfig, ViTEncoderModel
    torch.manual_seed(4)
    c = ViTConfig(image_size=(32, 32), patch_size=16, hidden_size=64, num_hidden_layers=2, num_attention_heads=2,
                  intermediate_size=128)
    m = ViTEncoderModel(c).eval()
    for p in m.parameters():
        torch.nn.init.normal_(p, std=0.05)
    px = torch.randn(2, 32, 32, 3).bfloat16()
    old, old_min = vit.NORM_HANDOFF, ops.FOLD_MIN_TILES
    try:
        ops.FOLD_MIN_TILES = 0
        vit.NORM_HANDOFF = True
        y1 = m(px)
        vit.NORM_HANDOFF = False
        y0 = m(px)
    finally:
        vit.NORM_HANDOFF, ops.FOLD_MIN_TILES = old, old_min
    assert rel(y1, y0) < 1e-2


def test_vit_cls_only_last_layer_cpu():
    """Classification reads token 0 only: the last layer's query side for that token alone (folded and plain paths)
    equals token 0 of the full encoder."""
    from shai_amd.models import vit
    from shai_amd.models.vit import ViTConfig, ViTEncoderModel
    torch.manual_seed(6)
    c = ViTConfig(image_size=(32, 32), patch_size=16, hidden_size=64, num_hidden_layers=2, num_attention_heads=2,
                  intermediate_size=128)
    m = ViTEncoderModel(c).eval()
    for p in m.parameters():
        torch.nn.init.normal_(p, std=0.05)
    px = torch.randn(3, 32, 32, 3).bfloat16()
    old, old_min = vit.NORM_HANDOFF, ops.FOLD_MIN_TILES
    try:
        for handoff in (True, False):
            ops.FOLD_MIN_TILES = 0
            vit.NORM_HANDOFF = handoff
            full = m(px)
            cls = m(px, cls_only=True)
            assert cls.shape == (3, 1, 64)
            assert rel(cls[:, 0], full[:, 0]) < 1e-2
            m.cfg.num_detection_tokens = 2  # the tail form (YOLOS detection tokens), here the last two patch tokens
            det = m(px, det_only=True)
            m.cfg.num_detection_tokens = 0
            assert det.shape == (3, 2, 64) and rel(det, full[:, -2:]) < 1e-2
    finally:
        vit.NORM_HANDOFF, ops.FOLD_MIN_TILES = old, old_min


def test_up2_phase_weights_match_upsample_conv():
    """Upsample + 3x3 conv == 4 output-phase 2x2 convs over the source with summed weights (gemm_8ph.hip CONV 3)."""
    torch.manual_seed(3)
    for n, h, w, c, co in [(2, 4, 5, 8, 16), (1, 3, 3, 16, 8), (1, 1, 2, 8, 8)]:
        x = torch.randn(n, h, w, c)
        wp = ref.pack_conv_weight(torch.randn(co, c, 3, 3))
        b, temb = torch.randn(co), torch.randn(n, co)
        y0 = ref.conv2d(x, wp, b, 3, 3, 1, 1, True, temb=temb, act="silu")
        y1 = ref.conv2d_up2_phases(x, ops.pack_up2_phase_weight(wp, c), b, temb=temb, act="silu")
        assert y1.shape == (n, 2 * h, 2 * w, co)
        torch.testing.assert_close(y1, y0, atol=1e-4, rtol=1e-4)
    # bf16 packing: the fp32 sums round once
    wb = ref.pack_conv_weight(torch.randn(8, 8, 3, 3)).to(torch.bfloat16)
    assert ops.pack_up2_phase_weight(wb, 8).dtype == torch.bfloat16
