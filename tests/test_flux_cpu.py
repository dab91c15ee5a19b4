"""Flux.1 transformer (fused, modulation-hoisted implementation) vs the unfused
fp32 reference in tests/flux_reference.py, same diffusers-format weights."""
import torch

from flux_reference import flux_reference, random_flux_state_dict
from shai_amd.models.flux import FluxConfig, FluxTransformer2DModel, pack_latents, unpack_latents_nhwc
from shai_amd.weights import load_into


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-6)).item()


def _setup(B=2, h2=4, w2=6, Nt=8):
    c = FluxConfig.tiny()
    sd = random_flux_state_dict(c)
    m = FluxTransformer2DModel(c)
    load_into(m, {k: v.clone() for k, v in sd.items()}, m.convert_hf_state_dict, strict=True)
    torch.manual_seed(0)
    lat = torch.randn(B, h2 * w2, c.in_channels).to(torch.bfloat16)
    t5 = torch.randn(B, Nt, c.joint_attention_dim).to(torch.bfloat16)
    pooled = torch.randn(B, c.pooled_projection_dim).to(torch.bfloat16)
    t = torch.tensor([0.9, 0.35])[:B]
    g = torch.full((B,), 3.5)
    return c, sd, m, lat, t5, pooled, t, g, h2, w2


def test_flux_transformer_matches_reference():
    c, sd, m, lat, t5, pooled, t, g, h2, w2 = _setup()
    with torch.no_grad():
        ref = flux_reference(sd, c, lat, t5, pooled, t, g, h2, w2)
        out = m(lat, t5, pooled, t, g, img_hw=(h2, w2))
    assert out.shape == ref.shape
    assert _rel(out, ref) < 0.03, _rel(out, ref)


def test_flux_hoisted_modulations_per_step():
    """Modulations precomputed for all steps at once == per-step evaluation."""
    c, sd, m, lat, t5, pooled, t, g, h2, w2 = _setup(B=1)
    ts = torch.tensor([1.0, 0.6, 0.2])
    with torch.no_grad():
        mods = m.modulations(ts, torch.full((3,), 3.5), pooled.expand(3, -1).contiguous())
        cos, sin = m.rope(t5.shape[1], h2, w2, lat.device)
        ctx = m.context_embedder(t5)
        for s in range(3):
            a = m.forward_step(lat, ctx, mods[s:s + 1], cos, sin)
            b = flux_reference(sd, c, lat, t5, pooled, ts[s:s + 1], torch.full((1,), 3.5), h2, w2)
            assert _rel(a, b) < 0.03


def test_pack_unpack_roundtrip():
    x = torch.randn(2, 16, 8, 12)
    p = pack_latents(x)
    assert p.shape == (2, 24, 64)
    nhwc = unpack_latents_nhwc(p, 8, 12)
    assert torch.equal(nhwc, x.permute(0, 2, 3, 1))
