"""HIP kernel numerics vs plain-PyTorch fp32 references (same random inputs).

Each test runs the native gfx950 kernel (torch.ops.shai.*) and the fp32 torch
reference from shai_amd.ops.reference and compares with bf16 tolerances.
"""
import math

import pytest
import torch

import shai_amd.ops as ops
from shai_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


def rnd(*shape, scale=1.0, device="cuda"):
    return (torch.randn(*shape, device=device) * scale).to(torch.bfloat16)


def close(a, b, atol, rtol=2e-2):
    a = a.float()
    b = b.float()
    err = (a - b).abs()
    tol = atol + rtol * b.abs()
    bad = (err > tol).float().mean().item()
    assert torch.isfinite(a).all(), "non-finite output"
    assert bad < 1e-3, f"{bad*100:.3f}% elements out of tolerance; max err {err.max().item():.4g}"


@pytest.mark.parametrize("D", [320, 768, 4096, 1280, 5120])
def test_rmsnorm(cuda, D):
    torch.manual_seed(0)
    x, r, w = rnd(67, D), rnd(67, D), rnd(D)
    y, nr = ops.rmsnorm(x, w, 1e-6, residual=r)
    yr, nrr = ref.rmsnorm(x, w, 1e-6, residual=r)
    close(y, yr, 2e-2)
    close(nr, nrr, 1e-2)
    y2, _ = ops.rmsnorm(x, w, 1e-5)
    close(y2, ref.rmsnorm(x, w, 1e-5)[0], 2e-2)


@pytest.mark.parametrize("D", [64, 192, 320, 512, 640, 768, 1024, 3072])
def test_layernorm(cuda, D):
    """D <= 512 (multiple of 64) runs the 8-rows-per-wave kernel; 129 rows leave a partial wave."""
    torch.manual_seed(1)
    x, w, b = rnd(129, D, scale=3.0) + 1.0, rnd(D), rnd(D)
    close(ops.layernorm(x, w, b, 1e-5)[0], ref.layernorm(x, w, b, 1e-5)[0], 2e-2)
    close(ops.layernorm(x, None, None, 1e-6)[0], ref.layernorm(x, None, None, 1e-6)[0], 2e-2)
    r = rnd(129, D)
    y, nr = ops.layernorm(x, w, b, 1e-5, residual=r)
    yr, nrr = ref.layernorm(x, w, b, 1e-5, residual=r)
    close(y, yr, 2e-2)
    close(nr, nrr, 1e-2)


@pytest.mark.parametrize("N,HW,C,G", [(2, 4096, 320, 32), (1, 256, 1280, 32), (2, 64, 2560, 32), (1, 16384, 128, 32),
                                      (3, 100, 64, 32)])
def test_groupnorm(cuda, N, HW, C, G):
    torch.manual_seed(2)
    x = rnd(N, HW, C, scale=2.0) + 0.5
    g, b = rnd(C), rnd(C)
    sc, sh = ops.groupnorm_stats(x, g, b, G, 1e-5)
    scr, shr = ref.groupnorm_stats(x, g, b, G, 1e-5)
    torch.testing.assert_close(sc, scr, atol=1e-3, rtol=1e-3)
    torch.testing.assert_close(sh, shr, atol=1e-3, rtol=1e-3)
    close(ops.groupnorm_apply(x, sc, sh, True), ref.groupnorm_apply(x, scr, shr, True), 2e-2)


@pytest.mark.parametrize("N,HW,C1,C2", [(2, 4096, 320, 320), (3, 64, 1280, 640), (1, 1000, 640, 320), (8, 256, 64, 256)])
@pytest.mark.parametrize("fused", [True, False])
def test_groupnorm_two_source(cuda, N, HW, C1, C2, fused, monkeypatch):
    """GN of cat([x, x2], -1) read from the two sources (UNet up-block skip concat) with the
    finalize fused into the stats launch (ticket counters) or as its own kernel; repeated calls
    check that the tickets re-arm."""
    monkeypatch.setattr(ops, "_GN_FUSED", fused)
    torch.manual_seed(5)
    x, x2 = rnd(N, HW, C1, scale=2.0) + 0.5, rnd(N, HW, C2) - 0.25
    g, b = rnd(C1 + C2), rnd(C1 + C2)
    xc = torch.cat([x, x2], -1)
    scr, shr = ref.groupnorm_stats(xc, g, b, 32, 1e-5)
    for _ in range(3):
        sc, sh = ops.groupnorm_stats(x, g, b, 32, 1e-5, x2=x2)
        torch.testing.assert_close(sc, scr, atol=1e-3, rtol=1e-3)
        torch.testing.assert_close(sh, shr, atol=1e-3, rtol=1e-3)
    y = ops.groupnorm_apply(x, sc, sh, True, x2=x2)
    assert y.shape == (N, HW, C1 + C2)
    close(y, ref.groupnorm_apply(xc, scr, shr, True), 2e-2)
    if fused:
        assert int(ops._gn_tickets(x, N)[:N].abs().sum()) == 0  # re-armed


@pytest.mark.parametrize("M,N,K", [(256, 256, 256), (1000, 320, 1280), (77, 1024, 1024), (8192, 640, 320),
                                   (5, 4096, 4096), (300, 96, 72)])
@pytest.mark.parametrize("act", ["none", "silu", "gelu"])
def test_gemm(cuda, M, N, K, act):
    torch.manual_seed(3)
    x, w, b, r = rnd(M, K), rnd(N, K, scale=1 / math.sqrt(K)), rnd(N), rnd(M, N)
    close(ops.linear(x, w, b, act=act, residual=r), ref.linear(x, w, b, act, r), 2e-2)


def test_gemm_identity_asymmetric(cuda):
    """A = I with an asymmetric W catches row/col swaps in the C write."""
    M = N = K = 128
    a = torch.eye(M, device="cuda").to(torch.bfloat16)
    w = (torch.arange(N * K, device="cuda").float().view(N, K) % 17 - 8).to(torch.bfloat16)
    y = ops.linear(a, w)
    torch.testing.assert_close(y.float(), w.float().t(), atol=0, rtol=0)


@pytest.mark.parametrize("act", ["gelu", "silu"])
def test_gemm_glu(cuda, act):
    torch.manual_seed(4)
    M, N, K = 500, 2 * 640, 320
    x, w, b = rnd(M, K), rnd(N, K, scale=1 / math.sqrt(K)), rnd(N)
    close(ops.linear(x, w, b, act=act, glu=True), ref.linear(x, w, b, act, glu=True), 2e-2)


@pytest.mark.parametrize("case", ["plain", "bias", "residual_inplace", "strided_out"])
def test_gemm_library_path(cuda, case):
    """force_cfg=2000 pins the hipBLASLt candidate of the autotuner (plain / bias / in-place residual)."""
    torch.manual_seed(6)
    M, N, K = 1000, 640, 320
    x, w, b = rnd(M, K), rnd(N, K, scale=1 / math.sqrt(K)), rnd(N)
    if case == "plain":
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        close(ops.gemm_into(x, w, out, force_cfg=2000), ref.linear(x, w), 2e-2)
    elif case == "bias":
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        close(ops.gemm_into(x, w, out, b, force_cfg=2000), ref.linear(x, w, b), 2e-2)
    elif case == "residual_inplace":
        r = rnd(M, N)
        want = ref.linear(x, w, None, None, r)
        close(ops.gemm_into(x, w, r, residual=r, force_cfg=2000), want, 2e-2)
    else:
        buf = torch.zeros(M, 2 * N, device="cuda", dtype=torch.bfloat16)
        ops.gemm_into(x, w, buf[:, N:], b, force_cfg=2000)
        close(buf[:, N:], ref.linear(x, w, b), 2e-2)
        assert buf[:, :N].abs().sum().item() == 0
    with pytest.raises(RuntimeError):
        ops.gemm_into(x, w, torch.empty(M, N, device="cuda", dtype=torch.bfloat16), b, act="gelu", force_cfg=2000)


def test_bmm(cuda):
    torch.manual_seed(5)
    a, w = rnd(3, 200, 64), rnd(3, 150, 64)
    close(ops.bmm(a, w, 0.5), (torch.matmul(a.float(), w.float().transpose(1, 2)) * 0.5), 2e-2)


@pytest.mark.parametrize("cfg", [
    dict(N=2, H=32, W=32, C=320, Co=320, k=3, s=1, p=1),
    dict(N=1, H=16, W=16, C=640, Co=1280, k=3, s=2, p=1),
    dict(N=2, H=8, W=8, C=128, Co=64, k=1, s=1, p=0),
    dict(N=1, H=24, W=20, C=8, Co=320, k=3, s=1, p=1),
    dict(N=1, H=16, W=16, C=512, Co=3, k=3, s=1, p=1),
])
def test_conv2d(cuda, cfg):
    torch.manual_seed(6)
    x = rnd(cfg["N"], cfg["H"], cfg["W"], cfg["C"])
    w = ops.pack_conv_weight(rnd(cfg["Co"], cfg["C"], cfg["k"], cfg["k"], scale=1 / math.sqrt(cfg["C"] * 9)))
    b = rnd(cfg["Co"])
    y = ops.conv2d(x, w, b, cfg["k"], cfg["k"], cfg["s"], cfg["p"])
    yr = ref.conv2d(x, w, b, cfg["k"], cfg["k"], cfg["s"], cfg["p"])
    close(y, yr, 3e-2)


def test_conv2d_fused(cuda):
    """GroupNorm+SiLU prologue, concat, upsample, temb bias and residual epilogue."""
    torch.manual_seed(7)
    N, H, W, C1, C2, Co = 2, 16, 16, 320, 640, 320
    x, x2 = rnd(N, H, W, C1), rnd(N, H, W, C2)
    sc, sh = ops.groupnorm_stats(torch.cat([x, x2], -1), rnd(C1 + C2), rnd(C1 + C2), 32, 1e-5)
    w = ops.pack_conv_weight(rnd(Co, C1 + C2, 3, 3, scale=1 / math.sqrt((C1 + C2) * 9)))
    b, temb = rnd(Co), rnd(N, Co)
    res = rnd(N, 2 * H, 2 * W, Co)
    y = ops.conv2d(x, w, b, 3, 3, 1, 1, upsample=True, x2=x2, norm=(sc, sh, "silu"), temb=temb, residual=res)
    yr = ref.conv2d(x, w, b, 3, 3, 1, 1, upsample=True, x2=x2, norm=(sc, sh, "silu"), temb=temb, residual=res)
    close(y, yr, 3e-2)


@pytest.mark.parametrize("N,H,W,C,Co,act", [(2, 16, 16, 1280, 1280, None), (3, 32, 32, 640, 640, "silu"),
                                            (1, 16, 32, 320, 320, None), (2, 32, 16, 128, 512, None),
                                            (8, 8, 8, 640, 640, "silu"), (4, 8, 16, 128, 256, None)])
def test_conv2d_upsample_phases(cuda, N, H, W, C, Co, act):
    """Phase-decomposed upsample conv (v4 CONV 3, 2x2 phase weights over the source) vs the fp32 upsample + 3x3
    conv, incl. the per-image bias, activation and the output's GroupNorm partials (per-image sums)."""
    torch.manual_seed(17)
    x = rnd(N, H, W, C)
    w = ops.pack_conv_weight(rnd(Co, C, 3, 3, scale=1 / math.sqrt(C * 9)))
    b = rnd(Co)
    temb = rnd(N, Co) if H * W >= 256 else None  # image groups (H W < 256) take no per-image bias
    assert ops.up2_phases_ok(x, 3, 3, 1, 1, temb=temb)
    assert not ops.up2_phases_ok(x, 3, 3, 1, 1, cout=Co)  # too small to leave the split-K 9-tap conv in a model
    wph = ops.pack_up2_phase_weight(w, C)
    y, gp = ops.conv2d(x, w, b, 3, 3, 1, 1, upsample=True, temb=temb, act=act, stats="gn", w_up2=wph)
    yr = ref.conv2d(x, w, b, 3, 3, 1, 1, upsample=True, temb=temb, act=act)
    close(y, yr, 3e-2)
    close(y, ref.conv2d_up2_phases(x, wph, b, temb, act), 2e-2)
    assert gp is not None
    want = ref.col_partials(y.reshape(-1, Co)).reshape(N, -1, Co, 2).sum(1)
    torch.testing.assert_close(gp.reshape(N, -1, Co, 2).sum(1), want, atol=2e-1, rtol=1e-3)
    # the plain (9-tap) path agrees
    close(ops.conv2d(x, w, b, 3, 3, 1, 1, upsample=True, temb=temb, act=act), yr, 3e-2)


@pytest.mark.parametrize("B,Sq,Skv,Hq,Hkv,D,causal", [
    (2, 256, 256, 4, 4, 64, False),
    (1, 1000, 77, 5, 5, 64, False),
    (2, 333, 333, 8, 2, 128, True),
    (1, 128, 128, 32, 8, 128, True),
    (3, 197, 197, 12, 12, 64, False),
    (1, 1056, 1056, 3, 3, 128, False),
    # d64, Sq not a multiple of the query tile (partial last workgroup), causal, GQA
    (2, 1030, 1030, 4, 2, 64, True),
    (1, 600, 77, 5, 5, 64, False),
    (2, 4096, 4096, 1, 1, 64, False),
])
def test_flash_attn(cuda, B, Sq, Skv, Hq, Hkv, D, causal):
    torch.manual_seed(8)
    q, k, v = rnd(B, Sq, Hq, D), rnd(B, Skv, Hkv, D), rnd(B, Skv, Hkv, D)
    o = ops.attention(q, k, v, causal=causal)
    orf = ref.attention(q, k, v, 1 / math.sqrt(D), causal)
    close(o, orf, 2e-2)


def test_flash_attn_strided_qkv_and_lens(cuda):
    torch.manual_seed(9)
    B, S, H, D = 3, 150, 12, 64
    qkv = rnd(B, S, 3, H, D)
    q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
    lens = torch.tensor([150, 77, 5], device="cuda", dtype=torch.int32)
    o = ops.attention(q, k, v, kv_lens=lens)
    orf = ref.attention(q, k, v, 1 / math.sqrt(D), kv_lens=lens)
    close(o, orf, 2e-2)


def test_flash_attn_bias(cuda):
    torch.manual_seed(10)
    B, S, H, D = 2, 96, 4, 64
    q, k, v = rnd(B, S, H, D), rnd(B, S, H, D), rnd(B, S, H, D)
    bias = rnd(H, S, S, scale=2.0)
    close(ops.attention(q, k, v, scale=1.0, bias=bias), ref.attention(q, k, v, 1.0, bias=bias), 3e-2)


@pytest.mark.parametrize("S,D", [(256, 128), (700, 64)])
def test_flash_attn_spike_forces_rescale(cuda, S, D):
    """Late keys with huge scores force the online-softmax rescale branch; a moderate one exercises the
    deferred-max path (row max grows by less than the threshold, no rescale)."""
    torch.manual_seed(11)
    B, H = 1, 2
    q, k, v = rnd(B, S, H, D), rnd(B, S, H, D), rnd(B, S, H, D)
    k[:, 200] = q[:, 10] * 4
    k[:, S - 3] = q[:, S - 40] * 4
    k[:, S // 2 + 1] = q[:, 30] * 0.6   # max growth below the deferred-rescale threshold (P up to 2^8)
    close(ops.attention(q, k, v), ref.attention(q, k, v, 1 / math.sqrt(D)), 2e-2)


@pytest.mark.parametrize("D", [64, 128])
def test_flash2_spike_late_and_first_tile(cuda, D):
    """flash2 (Sq >= 512): a huge score in the first tile, late spikes past the fast-path sum bound (exact
    path: tile max + O / l rescale) and a moderate growth that stays on the max-free fast path."""
    torch.manual_seed(13)
    B, S, H = 2, 1100, 2
    q, k, v = rnd(B, S, H, D), rnd(B, S, H, D), rnd(B, S, H, D)
    k[:, 3] = q[:, 700] * 3
    k[:, 900] = q[:, 10] * 5
    k[:, S - 2] = q[:, S - 300] * 5
    k[:, 513] = q[:, 600] * 0.7
    close(ops.attention(q, k, v), ref.attention(q, k, v, 1 / math.sqrt(D)), 2e-2)


@pytest.mark.parametrize("D,causal", [(64, False), (128, True), (64, True)])
def test_flash2_varlen_strided_gqa(cuda, D, causal):
    """flash2 with packed (strided) q/k/v rows, per-batch q / kv lengths and GQA 4:1."""
    torch.manual_seed(14)
    B, S, Hq, Hkv = 3, 777, 8, 2
    qkv = rnd(B, S, Hq + 2 * Hkv, D)
    q, k, v = qkv[:, :, :Hq], qkv[:, :, Hq:Hq + Hkv], qkv[:, :, Hq + Hkv:]
    kl = torch.tensor([777, 600, 65], device="cuda", dtype=torch.int32)
    ql = kl.clone() if causal else None
    o = ops.attention(q, k, v, causal=causal, kv_lens=kl, q_lens=ql)
    orf = ref.attention(q, k, v, 1 / math.sqrt(D), causal, 0, kl, ql)
    for b in range(B):  # rows past q_len are unspecified
        n = int((ql if ql is not None else torch.full_like(kl, S))[b])
        close(o[b, :n], orf[b, :n], 2e-2)


@pytest.mark.parametrize("causal", [False, True])
def test_flash2_d64_long_spikes_varlen(cuda, causal):
    """flash2 at D = 64 (Sq, Skv >= 2048: the SD2.1 self-attention kernel, pre-scaled Q and max-folded score
    accumulators): spikes in the first tile and past the fast-path bound, a moderate max growth, per-batch
    lengths with a partial last query tile, GQA 2:1."""
    torch.manual_seed(16)
    B, S, Hq, Hkv, D = 2, 2200, 4, 2, 64
    q, k, v = rnd(B, S, Hq, D), rnd(B, S, Hkv, D), rnd(B, S, Hkv, D)
    k[:, 3] = q[:, 700, :Hkv] * 3
    k[:, 1500] = q[:, 10, :Hkv] * 5
    k[:, S - 2] = q[:, S - 300, :Hkv] * 5
    k[:, 1025] = q[:, 600, :Hkv] * 0.7
    kl = torch.tensor([2200, 2090], device="cuda", dtype=torch.int32)
    ql = kl.clone() if causal else None
    o = ops.attention(q, k, v, causal=causal, kv_lens=kl, q_lens=ql)
    orf = ref.attention(q, k, v, 1 / math.sqrt(D), causal, 0, kl, ql)
    for b in range(B):
        n = int((ql if ql is not None else torch.full_like(kl, S))[b])
        close(o[b, :n], orf[b, :n], 2e-2)


@pytest.mark.parametrize("causal", [False, True])
def test_flash64_x2_large_grid(cuda, causal):
    """D = 64 launches of >= 1024 256-query workgroups run the two-group kernel (flash64x2, attention3.hip):
    spikes in the first tile and past the fast-path bound, per-batch lengths with partial query / key tiles,
    GQA 4:1 -- against the fp32 reference."""
    torch.manual_seed(17)
    B, S, Hq, Hkv, D = 8, 1100, 32, 8, 64
    q, k, v = rnd(B, S, Hq, D), rnd(B, S, Hkv, D), rnd(B, S, Hkv, D)
    k[:, 3] = q[:, 700, :Hkv] * 3
    k[:, 900] = q[:, 10, :Hkv] * 5
    k[:, 513] = q[:, 600, :Hkv] * 0.7
    kl = torch.tensor([1100, 1090, 1024, 777, 300, 1100, 65, 1000], device="cuda", dtype=torch.int32)
    ql = kl.clone() if causal else None
    o = ops.attention(q, k, v, causal=causal, kv_lens=kl, q_lens=ql)
    orf = ref.attention(q, k, v, 1 / math.sqrt(D), causal, 0, kl, ql)
    for b in range(B):
        n = int((ql if ql is not None else torch.full_like(kl, S))[b])
        close(o[b, :n], orf[b, :n], 2e-2)


def test_flash2_causal_offset_chunk(cuda):
    """Chunked-prefill shape: 600 new queries attending causally over 1500 keys (offset 900)."""
    torch.manual_seed(15)
    B, Sq, Skv, H, D = 1, 600, 1500, 4, 128
    q, k, v = rnd(B, Sq, H, D), rnd(B, Skv, H, D), rnd(B, Skv, H, D)
    o = ops.attention(q, k, v, causal=True, causal_offset=Skv - Sq)
    close(o, ref.attention(q, k, v, 1 / math.sqrt(D), True, Skv - Sq), 2e-2)


def test_flash_attn_bias_d64_long(cuda):
    torch.manual_seed(12)
    B, S, H, D = 1, 520, 2, 64
    q, k, v = rnd(B, S, H, D), rnd(B, S, H, D), rnd(B, S, H, D)
    bias = rnd(H, S, S, scale=2.0)
    close(ops.attention(q, k, v, scale=1.0, bias=bias), ref.attention(q, k, v, 1.0, bias=bias), 3e-2)


@pytest.mark.parametrize("S", [1000, 4096])
def test_attention_d512_vae(cuda, S):
    """The VAE mid-block attention (one head, D = 512) on the fused attention3.hip kernel against the fp32
    reference: q / k / v are strided views of one [B, S, 3 * 512] qkv tensor (as models/vae.py passes them),
    S = 1000 exercises the key / query tails (tiles of 32 keys, workgroups of 128 queries)."""
    torch.manual_seed(31)
    B, C = 2, 512
    qkv = rnd(B, S, 3 * C)
    q, k, v = (qkv[..., i * C:(i + 1) * C].view(B, S, 1, C) for i in range(3))
    sc = 1.0 / math.sqrt(C)
    o = ops.attention(q, k, v, scale=sc)
    close(o, ref.attention(q, k, v, sc), 2e-2)
    # a query row aligned with one key: the softmax is dominated by it (exercises the deferred-max rescale)
    k2 = k.clone()
    k2[0, S // 2, 0] = (q[0, 7, 0].float() * 3.0).to(torch.bfloat16)
    close(ops.attention(q, k2, v, scale=sc), ref.attention(q, k2, v, sc), 2e-2)


def _paged_setup(B, Hkv, D, ctx, nblocks=64):
    kc = rnd(nblocks, Hkv, 64, D)
    vc = rnd(nblocks, Hkv, 64, D)
    maxb = max((c + 63) // 64 for c in ctx)
    perm = torch.randperm(nblocks, device="cuda").to(torch.int32)
    bt = torch.zeros(B, maxb, dtype=torch.int32, device="cuda")
    i = 0
    for b, c in enumerate(ctx):
        nb = (c + 63) // 64
        bt[b, :nb] = perm[i:i + nb]
        i += nb
    return kc, vc, bt


@pytest.mark.parametrize("D,Hq,Hkv", [(128, 32, 8), (64, 8, 8), (128, 64, 8), (128, 16, 8), (64, 16, 4)])
@pytest.mark.parametrize("long_ctx", [False, True])
def test_decode_attn(cuda, D, Hq, Hkv, long_ctx):
    """Paged decode attention (LDS-DMA two-slot ring per 64-token block); long_ctx puts > 64 blocks
    in one split (block-id read-ahead reloads its 64-entry chunk)."""
    torch.manual_seed(12)
    ctx = [1, 64, 300, 1000] + ([4100, 5000] if long_ctx else [])
    B = len(ctx)
    kc, vc, bt = _paged_setup(B, Hkv, D, ctx, nblocks=sum((c + 63) // 64 for c in ctx) + 8)
    q = rnd(B, Hq, D)
    lens = torch.tensor(ctx, dtype=torch.int32, device="cuda")
    for splits in (1, 3):
        o = ops.decode_attention(q, kc, vc, bt, lens, num_splits=splits)
        close(o, ref.decode_attention(q, kc, vc, bt, lens, 1 / math.sqrt(D)), 2e-2)


@pytest.mark.parametrize("ctx", [[65536 + 17], [127744, 65600]])
def test_decode_attn_long_context_64k_128k(cuda, ctx):
    """Split-K paged decode attention at the reference's configured context (max_model_len 128000,
    cova/mllama-32-11b-vllm-trn1-config.yaml:12-16), Llama-3 GQA shape (32 q / 8 kv heads, D 128): the tuned
    split count (decode_splits), the cap (64) and an uneven one against the fp32 reference.  A "needle" key
    aligned with q far into the context (and one near the start) dominates each row's softmax, so a split that
    drops, double-counts or mis-rescales its partial shows up as a wrong output, not as averaged noise."""
    torch.manual_seed(21)
    D, Hq, Hkv = 128, 32, 8
    B = len(ctx)
    nblocks = sum((c + 63) // 64 for c in ctx) + 4
    kc, vc, bt = _paged_setup(B, Hkv, D, ctx, nblocks=nblocks)
    q = rnd(B, Hq, D)
    G = Hq // Hkv
    for b, c in enumerate(ctx):
        for pos in (5, c - 1000):
            blk, off = int(bt[b, pos // 64]), pos % 64
            for h in range(Hkv):   # key aligned with the group's first q head: score ~ 0.35 |q|^2 / sqrt(D)
                kc[blk, h, off] = (q[b, h * G].float() * 0.35).to(torch.bfloat16)
    lens = torch.tensor(ctx, dtype=torch.int32, device="cuda")
    want = ref.decode_attention(q, kc, vc, bt, lens, 1 / math.sqrt(D))
    for splits in (None, 64, 37):
        o = ops.decode_attention(q, kc, vc, bt, lens, num_splits=splits, max_ctx=max(ctx))
        close(o, want, 2e-2)


def test_paged_prefill_attn(cuda):
    torch.manual_seed(13)
    D, Hq, Hkv = 128, 8, 2
    ctx = [100, 300]
    q_lens = [37, 300]
    kc, vc, bt = _paged_setup(2, Hkv, D, ctx)
    q = rnd(2, 300, Hq, D)
    kl = torch.tensor(ctx, dtype=torch.int32, device="cuda")
    ql = torch.tensor(q_lens, dtype=torch.int32, device="cuda")
    o = ops.paged_attention(q, kc, vc, bt, kl, ql)
    orf = ref.paged_attention(q, kc, vc, bt, kl, ql, 1 / math.sqrt(D))
    close(o[0, :37], orf[0, :37], 2e-2)
    close(o[1], orf[1], 2e-2)


def test_kv_write(cuda):
    torch.manual_seed(14)
    T, H, D = 70, 8, 128
    k, v = rnd(T, H, D), rnd(T, H, D)
    kc, vc = torch.zeros(4, H, 64, D, dtype=torch.bfloat16, device="cuda"), torch.zeros(4, H, 64, D,
                                                                                      dtype=torch.bfloat16,
                                                                                      device="cuda")
    slots = torch.randperm(256, device="cuda")[:T].to(torch.int32)
    kr, vr = kc.clone(), vc.clone()
    ops.kv_write(k, v, kc, vc, slots)
    ref.kv_write(k, v, kr, vr, slots)
    assert torch.equal(kc, kr) and torch.equal(vc, vr)


def test_rope(cuda):
    torch.manual_seed(15)
    T, H, D = 33, 8, 128
    qkv = rnd(T, 3 * H * D)
    q = qkv[:, : H * D].view(T, H, D)
    pos = torch.randint(0, 500, (T,), device="cuda", dtype=torch.int32)
    inv = 1.0 / (10000 ** (torch.arange(0, D, 2, device="cuda").float() / D))
    fr = torch.outer(torch.arange(512, device="cuda").float(), inv)
    c, s = fr.cos().contiguous(), fr.sin().contiguous()
    qr = q.clone()
    ops.rope(q, pos, c, s)
    ref.rope(qr, pos, c, s, D)
    close(q, qr, 2e-2)


def test_rope_pairs(cuda):
    torch.manual_seed(16)
    B, T, H, D = 1, 40, 3, 128
    x = rnd(B, T, H, D)
    ang = torch.rand(T, D // 2, device="cuda") * 6
    xr = x.clone()
    ops.rope_pairs(x, ang.cos().contiguous(), ang.sin().contiguous())
    ref.rope_pairs(xr, ang.cos(), ang.sin())
    close(x, xr, 2e-2)


def test_gated_and_bias_act(cuda):
    torch.manual_seed(17)
    x = rnd(100, 2 * 1280)
    close(ops.gated_act(x, "gelu"), ref.gated_act(x, "gelu"), 2e-2)
    close(ops.gated_act(x, "silu", gate_first=True), ref.gated_act(x, "silu", True), 2e-2)
    y, b, r = rnd(64, 320), rnd(320), rnd(64, 320)
    close(ops.bias_act(y, b, r, "silu", 0.5), ref.bias_act(y, b, r, "silu", 0.5), 2e-2)


@pytest.mark.parametrize("pred", [0, 1, 2])
def test_sched_step(cuda, pred):
    torch.manual_seed(18)
    lat = rnd(2, 64, 64, 4)
    mo = rnd(4, 64, 64, 4)
    a = lat.clone()
    ops.sched_step(mo, lat, True, 7.5, pred, 0.5, 0.7, -0.05)
    ref.sched_step(mo, a, True, 7.5, pred, 0.5, 0.7, -0.05)
    close(lat, a, 3e-2)


def test_softmax_embedding(cuda):
    torch.manual_seed(19)
    x = rnd(10, 4096)
    y = x.clone()
    ops.softmax_(y, 0.125)
    close(y, torch.softmax(x.float() * 0.125, -1), 1e-3)
    table = rnd(1000, 256)
    ids = torch.randint(0, 1000, (3, 17), device="cuda")
    assert torch.equal(ops.embedding(ids, table), table[ids])


@pytest.mark.parametrize("M,N,K", [(256, 512, 8192), (64, 14336, 4096), (8, 4096, 4096), (1000, 320, 2880)])
def test_gemm_splitk_shapes(cuda, M, N, K):
    torch.manual_seed(20)
    x, w, b, r = rnd(M, K), rnd(N, K, scale=1 / math.sqrt(K)), rnd(N), rnd(M, N)
    close(ops.linear(x, w, b, act="silu", residual=r), ref.linear(x, w, b, "silu", r), 2e-2)


@pytest.mark.parametrize("cfg", [
    dict(N=8, H=8, W=8, C=1280, Co=1280),
    dict(N=2, H=16, W=16, C=2560, Co=1280),
])
def test_conv2d_small_spatial_splitk(cuda, cfg):
    torch.manual_seed(21)
    x = rnd(cfg["N"], cfg["H"], cfg["W"], cfg["C"])
    w = ops.pack_conv_weight(rnd(cfg["Co"], cfg["C"], 3, 3, scale=1 / math.sqrt(cfg["C"] * 9)))
    b, res = rnd(cfg["Co"]), rnd(cfg["N"], cfg["H"], cfg["W"], cfg["Co"])
    temb = rnd(cfg["N"], cfg["Co"])
    close(ops.conv2d(x, w, b, 3, 3, 1, 1, temb=temb, residual=res),
          ref.conv2d(x, w, b, 3, 3, 1, 1, temb=temb, residual=res), 3e-2)


@pytest.mark.parametrize("cfg", [2, 3, 4])  # 3 (128 x 128) keeps the separate fold
@pytest.mark.parametrize("splits", [2, 3, 5])
@pytest.mark.parametrize("M,N,K,glu", [(512, 1280, 2560, False), (130, 650, 1920, False), (512, 2560, 1280, True)])
def test_gemm2_splitk_fixup(cuda, cfg, splits, M, N, K, glu):
    """Split-K at the 64-128-column tiles, fixed up inside the launch (last-arriving K group sums the slabs in
    K-group order and runs the epilogue): vs fp32, and bit-identical across runs (arrival order does not matter)."""
    torch.manual_seed(22)
    x, w, b = rnd(M, K), rnd(N, K, scale=1 / math.sqrt(K)), rnd(N)
    r = rnd(M, N // 2 if glu else N)
    force = 3000 + 100 * splits + cfg
    out1 = torch.empty(M, N // 2 if glu else N, device="cuda", dtype=torch.bfloat16)
    out2 = torch.empty_like(out1)
    act = "gelu" if glu else "silu"
    ops.gemm_into(x, w, out1, b, act=act, residual=r, glu=glu, force_cfg=force)
    ops.gemm_into(x, w, out2, b, act=act, residual=r, glu=glu, force_cfg=force)
    close(out1, ref.linear(x, w, b, act, r, glu), 2e-2)
    assert torch.equal(out1, out2)


@pytest.mark.parametrize("causal", [False, True])
def test_flash128_x2_spikes_varlen_gqa(cuda, causal):
    """D = 128 two-group kernel (flash128x2, attention3.hip; opt-in for D = 128 at Sq, Skv >= 512): spikes in the
    first tile and past the fast-path bound, a moderate max growth, per-batch lengths with partial query / key tiles,
    GQA 4:1 -- against the fp32 reference, and against the flash2 kernel it replaced."""
    torch.manual_seed(18)
    B, S, Hq, Hkv, D = 3, 1100, 8, 2, 128
    q, k, v = rnd(B, S, Hq, D), rnd(B, S, Hkv, D), rnd(B, S, Hkv, D)
    k[:, 3] = q[:, 700, :Hkv] * 3
    k[:, 900] = q[:, 10, :Hkv] * 5
    k[:, 513] = q[:, 600, :Hkv] * 0.7
    kl = torch.tensor([1100, 1030, 513], device="cuda", dtype=torch.int32)
    ql = kl.clone() if causal else None
    K = ops._K()
    prev = K.set_flash128x2(1)
    try:
        o = ops.attention(q, k, v, causal=causal, kv_lens=kl, q_lens=ql)
        K.set_flash128x2(0)
        o2 = ops.attention(q, k, v, causal=causal, kv_lens=kl, q_lens=ql)
    finally:
        K.set_flash128x2(prev)
    orf = ref.attention(q, k, v, 1 / math.sqrt(D), causal, 0, kl, ql)
    for b in range(B):
        n = int((ql if ql is not None else torch.full_like(kl, S))[b])
        close(o[b, :n], orf[b, :n], 2e-2)
        close(o[b, :n], o2[b, :n], 2e-2)


@pytest.mark.parametrize("fused", [False, True])
def test_decode_attn_wave_per_block_matches_split_kernel(cuda, fused):
    """The short-context wave-per-block decode kernel (D 128, GQA 4, one split; each wave walks its own 64-token
    blocks for all four q heads) against the fp32 reference and the split kernel (set_decode_wb(0)): contexts of
    1 / 63 / 64 / 65 / 256 / 257 tokens (waves with no block, a ragged last block, more than one block per wave) and
    one of 17,000 (67 blocks per wave: the block-id read-ahead reloads its 64-entry chunk).  fused: RoPE + this
    step's k / v from the QKV rows (written to the cache, attended from registers), padding row (slot -1) last."""
    torch.manual_seed(31)
    D, Hq, Hkv = 128, 32, 8
    ctx = [1, 63, 64, 65, 256, 257, 17000, 5]
    B = len(ctx)
    kc, vc, bt = _paged_setup(B, Hkv, D, ctx, nblocks=sum((c + 63) // 64 for c in ctx) + 8)
    lens = torch.tensor(ctx, dtype=torch.int32, device="cuda")
    prev = ops.set_decode_wb(-1)
    try:
        if not fused:
            q = rnd(B, Hq, D)
            want = ref.decode_attention(q, kc, vc, bt, lens, 1 / math.sqrt(D))
            ops.set_decode_wb(1)
            o = ops.decode_attention(q, kc, vc, bt, lens, num_splits=1)
            ops.set_decode_wb(0)
            o_split = ops.decode_attention(q, kc, vc, bt, lens, num_splits=1)
            close(o, want, 2e-2)
            close(o, o_split, 2e-2)
            return
        qkv = rnd(B, (Hq + 2 * Hkv) * D)
        ang = torch.rand(max(ctx) + 1, D // 2, device="cuda") * 3
        cos, sin = ang.cos().contiguous(), ang.sin().contiguous()
        pos = lens - 1
        slots = torch.stack([bt[b, (c - 1) // 64] * 64 + (c - 1) % 64 for b, c in enumerate(ctx)]).int()
        slots[-1] = -1
        outs, caches = [], []
        for mode in (1, 0):
            ops.set_decode_wb(mode)
            k2, v2 = kc.clone(), vc.clone()
            outs.append(ops.decode_attention_rope(qkv.clone(), k2, v2, bt, lens, pos, cos, sin, slots, Hq, Hkv,
                                                  num_splits=1))
            caches.append((k2, v2))
        assert torch.equal(caches[0][0], caches[1][0]) and torch.equal(caches[0][1], caches[1][1])
        close(outs[0][:-1], outs[1][:-1], 2e-2)
        # fp32 reference over the updated cache (the new token is in it now)
        q2 = qkv.clone()
        k3, v3 = kc.clone(), vc.clone()
        ops.rope_qkv_cache(q2, pos, cos, sin, k3, v3, slots, Hq, Hkv)
        want = ref.decode_attention(q2[:, :Hq * D].reshape(B, Hq, D), k3, v3, bt, lens, 1 / math.sqrt(D))
        close(outs[0][:-1], want.reshape(B, Hq * D)[:-1], 2e-2)
    finally:
        ops.set_decode_wb(prev)


def test_upsample2d_layer_takes_phase_conv_and_tracks_weight_updates(cuda):
    """Upsample2D (UNet / VAE) on a shape with >= 256 output tiles runs the phase conv with cached phase weights,
    matches the fp32 upsample + 3x3 conv, and rebuilds the phase weights after an in-place weight update."""
    from shai_amd.models.unet2d import Upsample2D
    torch.manual_seed(23)
    C = 64
    up = Upsample2D(C).to("cuda")
    with torch.no_grad():
        up.conv.weight.copy_(ops.pack_conv_weight(rnd(C, C, 3, 3, scale=1 / math.sqrt(C * 9))))
        up.conv.bias.copy_(rnd(C))
    x = rnd(16, 32, 32, C)
    assert ops.up2_phases_ok(x, 3, 3, 1, 1, cout=C)
    y = up(x)
    assert getattr(up.conv, "_w_up2", None) is not None, "phase conv not taken"
    close(y, ref.conv2d(x, up.conv.weight, up.conv.bias, 3, 3, 1, 1, upsample=True), 3e-2)
    with torch.no_grad():
        up.conv.weight.mul_(-0.5)
    y2 = up(x)
    close(y2, ref.conv2d(x, up.conv.weight, up.conv.bias, 3, 3, 1, 1, upsample=True), 3e-2)


@pytest.mark.parametrize("S,R,N,K", [(4, 256, 320, 320), (2, 1024, 640, 640), (8, 512, 256, 192)])
def test_linear_weight_slices(cuda, S, R, N, K):
    """One GEMM whose row blocks of R rows each take their own weight slice and bias row (v4 kernel, w_slice_rows),
    with the output's LayerNorm (mean, rstd) from the epilogue."""
    torch.manual_seed(31)
    x, w, b2 = rnd(S * R, K), rnd(S, N, K, scale=1 / math.sqrt(K)), rnd(S, N)
    y, st = ops.linear_wslices(x, w, b2, R, stats="ln", eps=1e-5)
    want = torch.einsum("smk,snk->smn", x.float().view(S, R, K), w.float()) + b2.float()[:, None, :]
    close(y, want.reshape(S * R, N), 2e-2)
    torch.testing.assert_close(st, ref.row_moments(y, 1e-5), atol=2e-3, rtol=2e-3)
