"""W-stationary low-K GEMM (csrc/kernels/gemm_ws.hip, tuner config 15) vs fp32 PyTorch, forced for every epilogue it
implements: bias / activation / residual (BM = 32 tiles), GLU (erf / tanh GELU, SiLU), the folded LayerNorm (with a
large per-row DC offset), ragged M (partial last tile, prefetches past the end), several 320-column N slices."""
import pytest
import torch

from shai_amd import ops

pytestmark = pytest.mark.gpu
WS = 15


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-6)).item()


@pytest.mark.parametrize("M,N", [(65536, 320), (1000, 960), (4099, 2560), (64, 640), (17, 320)])
@pytest.mark.parametrize("act", [None, "silu", "gelu"])
def test_ws_bias_act(cuda, M, N, act):
    K = 320
    torch.manual_seed(M + N)
    a = torch.randn(M, K, device=cuda).bfloat16()
    w = (torch.randn(N, K, device=cuda) / K ** 0.5).bfloat16()
    b = torch.randn(N, device=cuda).bfloat16()
    out = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
    ops.gemm_into(a, w, out, b, act=act, force_cfg=WS)
    y = a.float() @ w.float().t() + b.float()
    if act == "silu":
        y = torch.nn.functional.silu(y)
    elif act == "gelu":
        y = torch.nn.functional.gelu(y)
    assert _rel(out, y) < 1e-2


@pytest.mark.parametrize("M,N", [(262144, 320), (1000, 640), (33, 320)])
def test_ws_residual_inplace(cuda, M, N):
    """out = x W^T + b + res_alpha * R with the residual tile staged next to A (BM = 32); in place (C aliases R)."""
    K = 320
    torch.manual_seed(7)
    a = torch.randn(M, K, device=cuda).bfloat16()
    w = (torch.randn(N, K, device=cuda) / K ** 0.5).bfloat16()
    b = torch.randn(N, device=cuda).bfloat16()
    r = torch.randn(M, N, device=cuda).bfloat16()
    want = a.float() @ w.float().t() + b.float() + 0.5 * r.float()
    ops.gemm_into(a, w, r, b, residual=r, res_alpha=0.5, force_cfg=WS)
    assert _rel(r, want) < 1e-2


@pytest.mark.parametrize("act", ["gelu", "silu", "gelu_tanh"])
@pytest.mark.parametrize("M", [262144, 999])
def test_ws_glu(cuda, act, M):
    K, N = 320, 2560
    torch.manual_seed(3)
    a = torch.randn(M, K, device=cuda).bfloat16()
    w = (torch.randn(N, K, device=cuda) / K ** 0.5).bfloat16()
    b = torch.randn(N, device=cuda).bfloat16()
    out = torch.empty(M, N // 2, device=cuda, dtype=torch.bfloat16)
    ops.gemm_into(a, w, out, b, act=act, glu=True, force_cfg=WS)
    y = a.float() @ w.float().t() + b.float()
    f = {"gelu": torch.nn.functional.gelu, "silu": torch.nn.functional.silu,
         "gelu_tanh": lambda t: torch.nn.functional.gelu(t, approximate="tanh")}[act]
    assert _rel(out, y[:, 0::2] * f(y[:, 1::2])) < 1e-2


@pytest.mark.parametrize("glu,res", [(False, False), (True, False), (False, True)])
def test_ws_folded_layernorm(cuda, glu, res):
    """LayerNorm(x) @ W^T + b as rstd * (x @ W'^T - mean * s) + b' (ops.fold_layernorm) on the W-stationary kernel,
    rows with a large DC offset (|mean| / std = 20), against the fp32 LayerNorm + GEMM."""
    M, K = 4096 + 40, 320
    N = 2560 if glu else 960
    torch.manual_seed(11)
    x = (torch.randn(M, K, device=cuda) + 20.0 * torch.randn(M, 1, device=cuda)).bfloat16()
    w = (torch.randn(N, K, device=cuda) / K ** 0.5).bfloat16()
    b = torch.randn(N, device=cuda).bfloat16()
    g = (1 + 0.1 * torch.randn(K, device=cuda)).bfloat16()
    be = (0.1 * torch.randn(K, device=cuda)).bfloat16()
    xf = x.float()
    mean = xf.mean(1)
    rstd = torch.rsqrt(xf.var(1, unbiased=False) + 1e-5)
    mr = torch.stack([mean, rstd], 1).contiguous()
    w2, b2, s = ops.fold_layernorm(w, b, g, be)
    r = torch.randn(M, N, device=cuda).bfloat16() if res else None
    y = ops.linear(x, w2, b2, act="gelu" if glu else None, glu=glu, residual=r, row_affine=(mr, s), force_cfg=WS)
    ln = torch.nn.functional.layer_norm(xf, (K,), g.float(), be.float(), 1e-5)
    want = ln @ w.float().t() + b.float()
    if glu:
        want = want[:, 0::2] * torch.nn.functional.gelu(want[:, 1::2])
    if res:
        want = want + r.float()
    assert _rel(y, want) < 2e-2


_ACTS = {None: lambda t: t, "silu": torch.nn.functional.silu, "gelu": torch.nn.functional.gelu,
         "gelu_tanh": lambda t: torch.nn.functional.gelu(t, approximate="tanh"),
         "quick_gelu": lambda t: t * torch.sigmoid(1.702 * t), "relu": torch.relu}


@pytest.mark.parametrize("act,glu", [("relu", False), ("gelu_tanh", False), ("quick_gelu", False), ("relu", True),
                                     ("quick_gelu", True), (None, True)])
def test_ws_rejects_uninstantiated_act(cuda, act, glu):
    """gemm_ws_supported() admits exactly the activation variants launch_gemm_ws instantiates: forcing config 15 on
    any other (act, glu) pair raises instead of silently running another activation."""
    M, K, N = 1024, 320, 640
    a = torch.randn(M, K, device=cuda).bfloat16()
    w = (torch.randn(N, K, device=cuda) / K ** 0.5).bfloat16()
    out = torch.empty(M, N // 2 if glu else N, device=cuda, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError, match="bad force_cfg"):
        ops.gemm_into(a, w, out, None, act=act, glu=glu, force_cfg=WS)


@pytest.mark.parametrize("act,glu", [("relu", False), ("gelu_tanh", False), ("quick_gelu", False), ("relu", True),
                                     ("quick_gelu", True), ("silu", True)])
def test_ws_shape_autotuned_any_act(cuda, act, glu):
    """The same K = 320 shapes autotuned (config 15 is a candidate only where supported, and a cached choice of
    another activation's problem falls back) match fp32 for every activation."""
    M, K, N = 8192, 320, 1280
    torch.manual_seed(5)
    a = torch.randn(M, K, device=cuda).bfloat16()
    w = (torch.randn(N, K, device=cuda) / K ** 0.5).bfloat16()
    b = torch.randn(N, device=cuda).bfloat16()
    # prime the tuning cache with the plain problem of this shape (config 15 may win it)
    ops.linear(a, w, b, act="gelu" if glu else None, glu=glu)
    y = ops.linear(a, w, b, act=act, glu=glu)
    f = _ACTS[act]
    ref = a.float() @ w.float().t() + b.float()
    want = ref[:, 0::2] * f(ref[:, 1::2]) if glu else f(ref)
    assert _rel(y, want) < 1e-2


@pytest.mark.parametrize("M", [262144, 1003])
def test_ws_lnout(cuda, M):
    """ops.linear_lnout: y = x W^T + b + R and LayerNorm(y) gamma + beta from the W-stationary epilogue (row moments
    across the 4 waves, two-pass) vs fp32 -- rows with a large DC offset, a ragged last tile."""
    K = N = 320
    torch.manual_seed(13)
    x = torch.randn(M, K, device=cuda).bfloat16()
    w = (torch.randn(N, K, device=cuda) / K ** 0.5).bfloat16()
    b = torch.randn(N, device=cuda).bfloat16()
    r = (torch.randn(M, N, device=cuda) + 30.0 * torch.randn(M, 1, device=cuda)).bfloat16()
    g = (1 + 0.1 * torch.randn(N, device=cuda)).bfloat16()
    be = (0.1 * torch.randn(N, device=cuda)).bfloat16()
    y, yn = ops.linear_lnout(x, w, b, r, g, be, 1e-5)
    # the fused kernel ran (not the GEMM + LayerNorm fallback)
    y2, yn2 = torch.empty_like(y), torch.empty_like(y)
    assert ops._K().gemm_lnout(x, w, y2, yn2, b, r, 1.0, g, be, 1e-5)
    assert torch.equal(y2, y) and torch.equal(yn2, yn)
    want = x.float() @ w.float().t() + b.float() + r.float()
    assert _rel(y, want) < 1e-2
    # the norm of the stored bf16 y (what a standalone LayerNorm of y reads)
    wn = torch.nn.functional.layer_norm(y.float(), (N,), g.float(), be.float(), 1e-5)
    assert _rel(yn, wn) < 1e-2
    assert (yn.float() - wn).abs().max().item() < 0.1
