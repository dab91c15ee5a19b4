"""Flux building-block kernels and the Flux transformer / engine on the MI355X,
against fp32 PyTorch references."""
import pytest
import torch

from shai_amd import ops
from shai_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-6)).item()


@pytest.mark.parametrize("B,M,N,K", [(1, 1536, 3072, 3072), (2, 300, 640, 256), (3, 77, 200, 64)])
def test_gemm_gated_residual_inplace(cuda, B, M, N, K):
    torch.manual_seed(0)
    x = torch.randn(B, M, K, device=cuda).bfloat16()
    w = (torch.randn(N, K, device=cuda) / K ** 0.5).bfloat16()
    b = torch.randn(N, device=cuda).bfloat16()
    mod = torch.randn(B, 3 * N, device=cuda).bfloat16()
    gate = mod[:, N:2 * N]
    res = torch.randn(B, M, N, device=cuda).bfloat16()
    want = res.float() + gate.float()[:, None] * (x.float() @ w.float().t() + b.float())
    out = res.clone()
    ops.gemm_into(x, w, out, b, residual=out, gate=gate, rows_per_gate=M)  # in place, autotuned on first call
    assert _rel(out, want) < 1e-2
    out2 = res.clone()
    ops.gemm_into(x, w, out2, b, residual=out2, gate=gate, rows_per_gate=M)  # cached config
    assert _rel(out2, want) < 1e-2


def test_gemm_strided_output_rows(cuda):
    """QKV GEMMs writing into the text / image row ranges of one joint buffer."""
    B, Nt, Ni, K, N = 2, 40, 96, 128, 384
    xt = torch.randn(B, Nt, K, device=cuda).bfloat16()
    xi = torch.randn(B, Ni, K, device=cuda).bfloat16()
    wt = torch.randn(N, K, device=cuda).bfloat16()
    wi = torch.randn(N, K, device=cuda).bfloat16()
    j = torch.zeros(B, Nt + Ni, N, device=cuda).bfloat16()
    ops.gemm_into(xt, wt, j[:, :Nt])
    ops.gemm_into(xi, wi, j[:, Nt:], act="gelu_tanh")
    assert _rel(j[:, :Nt], xt.float() @ wt.float().t()) < 1e-2
    assert _rel(j[:, Nt:], torch.nn.functional.gelu(xi.float() @ wi.float().t(), approximate="tanh")) < 1e-2


@pytest.mark.parametrize("D", [3072, 128])
def test_layernorm_mod(cuda, D):
    B, S = 2, 257
    x = torch.randn(B, S, D, device=cuda).bfloat16()
    mod = torch.randn(B, 6 * D, device=cuda).bfloat16()
    scale, shift = mod[:, D:2 * D], mod[:, :D]
    y = ops.layernorm_mod(x, scale, shift, S)
    want = ref.layernorm_mod(x.cpu(), scale.cpu(), shift.cpu(), S, 1e-6)
    assert _rel(y, want) < 1e-2


@pytest.mark.parametrize("H,D", [(24, 128), (2, 64)])
def test_qk_norm_rope(cuda, H, D):
    rows, S = 300, 150
    x = torch.randn(rows, 3 * H * D, device=cuda).bfloat16()
    qw = (1 + 0.1 * torch.randn(D, device=cuda)).bfloat16()
    kw = (1 + 0.1 * torch.randn(D, device=cuda)).bfloat16()
    ang = torch.rand(S, D // 2, device=cuda) * 6
    cos, sin = torch.cos(ang).contiguous(), torch.sin(ang).contiguous()
    want = ref.qk_norm_rope(x.cpu().clone(), qw.cpu(), kw.cpu(), cos.cpu(), sin.cpu(), H, D, S, 1e-6)
    got = ops.qk_norm_rope(x.clone(), qw, kw, cos, sin, H, D, S)
    assert _rel(got, want) < 1e-2
    assert torch.equal(got[:, 2 * H * D:].cpu(), x[:, 2 * H * D:].cpu())  # v untouched


def _small_cfg():
    from shai_amd.models.flux import FluxConfig
    return FluxConfig(hidden=256, heads=2, head_dim=128, num_layers=2, num_single_layers=2, joint_attention_dim=128,
                      pooled_projection_dim=64, axes_dims_rope=(16, 56, 56))


def test_flux_transformer_gpu_matches_reference(cuda):
    import sys, os
    sys.path.insert(0, os.path.dirname(__file__))
    from flux_reference import flux_reference, random_flux_state_dict
    from shai_amd.models.flux import FluxTransformer2DModel
    from shai_amd.weights import load_into
    c = _small_cfg()
    sd = random_flux_state_dict(c, seed=1)
    m = FluxTransformer2DModel(c)
    load_into(m, {k: v.clone() for k, v in sd.items()}, m.convert_hf_state_dict, strict=True)
    m = m.to(cuda)
    B, h2, w2, Nt = 2, 16, 16, 64
    torch.manual_seed(0)
    lat = torch.randn(B, h2 * w2, c.in_channels).bfloat16()
    t5 = torch.randn(B, Nt, c.joint_attention_dim).bfloat16()
    pooled = torch.randn(B, c.pooled_projection_dim).bfloat16()
    t = torch.tensor([0.8, 0.3])
    g = torch.full((B,), 3.5)
    with torch.no_grad():
        want = flux_reference(sd, c, lat, t5, pooled, t, g, h2, w2)
        got = m(lat.to(cuda), t5.to(cuda), pooled.to(cuda), t.to(cuda), g.to(cuda), img_hw=(h2, w2))
    assert _rel(got, want) < 0.04, _rel(got, want)


def test_flux_engine_graph_matches_eager(cuda):
    from shai_amd.engines.flux import FluxEngine, FluxPipelineConfig
    cfg = FluxPipelineConfig.tiny()
    cfg.transformer = _small_cfg()
    cfg.clip.hidden_size = cfg.transformer.pooled_projection_dim
    cfg.t5.d_model = cfg.transformer.joint_attention_dim
    eng = FluxEngine(cfg, device="cuda", use_graphs=True)
    a = eng.generate(["a fox", "a hen"], 4, seed=3, output="tensor").float()
    eng.use_graphs = False
    b = eng.generate(["a fox", "a hen"], 4, seed=3, output="tensor").float()
    assert torch.isfinite(a).all() and _rel(a, b) < 2e-2
