"""fp8 (OCP e4m3) weight-only path: native dequant vs torch's float8 conversion, the skinny
decode GEMM streaming fp8 weights vs fp32 PyTorch on the dequantised weights, and an fp8 LLM
engine decode vs the same engine in bf16."""
import pytest
import torch

from shai_amd import ops

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-6)).item()


def test_dequant_matches_torch_float8(cuda):
    torch.manual_seed(0)
    w = torch.randn(256, 512, device=cuda) * torch.rand(256, 1, device=cuda) * 3
    w8, sc = ops.quantize_fp8_rows(w)
    assert w8.dtype == torch.float8_e4m3fn and sc.shape == (256,)
    want = (w8.float() * sc[:, None]).bfloat16()     # torch's own e4m3fn decode
    got = ops.dequant_fp8(w8, sc)
    torch.testing.assert_close(got.float(), want.float(), atol=0, rtol=0)
    assert _rel(got, w) < 0.05                        # e4m3: 3 mantissa bits


@pytest.mark.parametrize("M,N,K", [(1, 4096, 4096), (8, 6144, 4096), (32, 4096, 14336), (33, 4096, 4096),
                                   (64, 28672, 4096), (5, 96, 64)])
def test_fp8_skinny_plain_residual(cuda, M, N, K):
    torch.manual_seed(M + N)
    x = torch.randn(M, K, device=cuda).bfloat16()
    w8, sc = ops.quantize_fp8_rows(torch.randn(N, K, device=cuda) / K ** 0.5)
    wd = w8.float() * sc[:, None]
    b = torch.randn(N, device=cuda).bfloat16()
    r = torch.randn(M, N, device=cuda).bfloat16()
    y = ops.linear(x, w8, b, residual=r, w_scale=sc)
    want = x.float() @ wd.t() + b.float() + r.float()
    assert _rel(y, want) < 1e-2


@pytest.mark.parametrize("M", [1, 17, 64])
def test_fp8_skinny_glu_rms(cuda, M):
    """SwiGLU gate/up (interleaved rows) with the RMSNorm folded in, as in Mistral decode."""
    torch.manual_seed(M)
    K, N = 4096, 2 * 1792
    x = torch.randn(M, K, device=cuda).bfloat16() * 3
    w8, sc = ops.quantize_fp8_rows(torch.randn(N, K, device=cuda) / K ** 0.5)
    wd = w8.float() * sc[:, None]
    y = ops.linear(x, w8, act="silu", glu=True, rms_eps=1e-5, w_scale=sc)
    xf = x.float()
    xn = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-5)
    h = xn @ wd.t()
    want = h[:, 0::2] * torch.nn.functional.silu(h[:, 1::2])
    assert _rel(y, want) < 2e-2


@pytest.mark.parametrize("cfg", [1004, 1104, 1108])
def test_fp8_skinny_forced_k_groups(cuda, cfg):
    """fp8 weights with split-K: separate fold (1000 + kg) and in-kernel fixup (1100 + kg), GLU + RMS."""
    torch.manual_seed(cfg)
    M, K, N = 48, 4096, 2 * 1024
    x = torch.randn(M, K, device=cuda).bfloat16() * 3
    w8, sc = ops.quantize_fp8_rows(torch.randn(N, K, device=cuda) / K ** 0.5)
    wd = w8.float() * sc[:, None]
    out = torch.empty(M, N // 2, device=cuda, dtype=torch.bfloat16)
    ops.gemm_into(x, w8, out, act="silu", glu=True, rms_eps=1e-5, w_scale=sc, force_cfg=cfg)
    xf = x.float()
    h = (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-5)) @ wd.t()
    assert _rel(out, h[:, 0::2] * torch.nn.functional.silu(h[:, 1::2])) < 2e-2


@pytest.mark.parametrize("mode", ["dequant", "w8a8"])
def test_fp8_large_m_prefill_paths(cuda, mode, monkeypatch):
    """Prefill-shaped problems (M > 64): "dequant" widens the weights to bf16 and runs the bf16 GEMMs (bf16
    accuracy); "w8a8" (the default) also quantises the activation rows to e4m3, so its error is that of two
    fp8 operands (about 2^-4 per element, ~3 % relative on the product)."""
    monkeypatch.setattr(ops, "FP8_PREFILL", mode)
    torch.manual_seed(3)
    x = torch.randn(300, 1024, device=cuda).bfloat16()
    w8, sc = ops.quantize_fp8_rows(torch.randn(512, 1024, device=cuda) / 32)
    y = ops.linear(x, w8, w_scale=sc)
    assert _rel(y, x.float() @ (w8.float() * sc[:, None]).t()) < (1e-2 if mode == "dequant" else 5e-2)


def test_fp8_llm_engine_decode(cuda):
    from shai_amd.engines.llm import LLMEngine, SamplingParams
    from shai_amd.models.llama import LlamaConfig
    c = LlamaConfig.tiny()
    e16 = LLMEngine(c, device=cuda, max_num_seqs=4, max_model_len=256, seed=1, enable_prefix_caching=False)
    e8 = LLMEngine(c, device=cuda, max_num_seqs=4, max_model_len=256, seed=1, enable_prefix_caching=False,
                   quantization="fp8")
    assert e8.model.layers[0].mlp.gate_up_proj.weight.dtype == torch.float8_e4m3fn
    prompts = [[3, 17, 99, 250, 7], [5, 6, 7, 8, 9, 10, 11]]
    p = SamplingParams(max_tokens=8, temperature=0.0, ignore_eos=True)
    o16 = [s.output for s in e16.generate(prompts, p)]
    o8 = [s.output for s in e8.generate(prompts, p)]
    assert all(len(o) == 8 for o in o8)
    # random-init weights: greedy continuations agree on the first tokens at least
    assert sum(a[0] == b[0] for a, b in zip(o16, o8)) >= 1
