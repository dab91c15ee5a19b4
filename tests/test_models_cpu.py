"""CPU-path tests of the diffusion stack (fp32 reference ops) and transformers parity for CLIP."""
import numpy as np
import pytest
import torch

from shai_amd import ops
from shai_amd.ops import reference as ref


def test_conv_pack_roundtrip():
    w = torch.randn(5, 8, 3, 3)
    assert torch.equal(ops.unpack_conv_weight(ops.pack_conv_weight(w), 8, 3, 3), w)


def test_conv_ref_matches_torch_nchw():
    x = torch.randn(2, 9, 7, 16)
    w = torch.randn(4, 16, 3, 3)
    y = ref.conv2d(x.double().float(), ops.pack_conv_weight(w), None, 3, 3, 2, 1)
    yt = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2), w, stride=2, padding=1).permute(0, 2, 3, 1)
    torch.testing.assert_close(y, yt, atol=1e-4, rtol=1e-4)


def test_sd_tiny_pipeline_cpu():
    from shai_amd.engines.diffusion import SDConfig, StableDiffusionEngine
    e = StableDiffusionEngine(SDConfig.tiny(), device="cpu")
    a = e(["a cat", "a dog"], num_inference_steps=3, seed=1)
    b = e(["a cat", "a dog"], num_inference_steps=3, seed=1)
    assert a.shape == (2, 64, 64, 3) and a.dtype == torch.uint8
    assert torch.equal(a, b)


def test_schedulers():
    from shai_amd.schedulers import DDIMScheduler, FlowMatchEulerScheduler
    st = DDIMScheduler().steps(50)
    assert len(st) == 50 and st[0].t == 981.0 and st[-1].t == 1.0
    assert st[-1].a_prev == pytest.approx(DDIMScheduler().alphas_cumprod[0])
    fm = FlowMatchEulerScheduler().steps(10, 1024)
    assert len(fm) == 10 and abs(sum(s.dt for s in fm) + 1.0) < 1e-6


def test_clip_matches_transformers():
    transformers = pytest.importorskip("transformers")
    from shai_amd.models.clip import CLIPTextConfig, CLIPTextModel
    from shai_amd.weights import load_into
    c = CLIPTextConfig.tiny()
    hc = transformers.CLIPTextConfig(vocab_size=c.vocab_size, hidden_size=c.hidden_size,
                                     intermediate_size=c.intermediate_size, num_hidden_layers=c.num_hidden_layers,
                                     num_attention_heads=c.num_attention_heads, max_position_embeddings=77,
                                     hidden_act="gelu", bos_token_id=c.bos_token_id, eos_token_id=c.eos_token_id)
    torch.manual_seed(0)
    hf = transformers.CLIPTextModel(hc).eval()
    with torch.no_grad():
        for p in hf.parameters():
            p.copy_(p.to(torch.bfloat16).float())
    m = CLIPTextModel(c)
    load_into(m, {k: v.clone() for k, v in hf.state_dict().items()}, CLIPTextModel.convert_hf_state_dict, strict=True)
    ids = torch.randint(0, 990, (2, 77))
    ids[:, 0] = c.bos_token_id
    ids[0, 10] = c.eos_token_id
    ids[1, 30] = c.eos_token_id
    with torch.no_grad():
        r = hf(ids)
        y, pooled = m(ids, output_pooled=True)
    assert ((y.float() - r.last_hidden_state).norm() / r.last_hidden_state.norm()) < 0.02
    assert ((pooled.float() - r.pooler_output).norm() / r.pooler_output.norm()) < 0.02


def test_flops_counter():
    from shai_amd.bench.flops import sd21_unet_flops
    fc = sd21_unet_flops(2)
    assert 1.4e12 < fc.total < 1.8e12


def test_linear_lnout_cpu_reference():
    """ops.linear_lnout on the CPU: (x W^T + b + R, LayerNorm of it) -- the contract the fused GPU epilogue meets."""
    import torch
    from shai_amd import ops
    torch.manual_seed(0)
    x, w, b = torch.randn(37, 320), torch.randn(320, 320) / 18, torch.randn(320)
    r, g, be = torch.randn(37, 320) + 5, 1 + 0.1 * torch.randn(320), 0.1 * torch.randn(320)
    y, yn = ops.linear_lnout(x, w, b, r, g, be, 1e-5)
    want = x @ w.t() + b + r
    assert torch.allclose(y, want, atol=1e-4)
    assert torch.allclose(yn, torch.nn.functional.layer_norm(want, (320,), g, be, 1e-5), atol=1e-4)
