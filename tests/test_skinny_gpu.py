"""Skinny (decode-shaped, M <= 32) streaming GEMM kernel vs fp32 PyTorch."""
import pytest
import torch

from shai_amd import ops

pytestmark = pytest.mark.gpu
SKINNY = 1000


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-6)).item()


@pytest.mark.parametrize("M,N,K", [(1, 4096, 4096), (7, 6144, 4096), (32, 4096, 14336), (32, 28672, 4096),
                                   (16, 1024, 512), (32, 32768, 4096), (3, 96, 64)])
def test_skinny_plain(cuda, M, N, K):
    torch.manual_seed(M + N)
    x = torch.randn(M, K, device=cuda).bfloat16()
    w = (torch.randn(N, K, device=cuda) / K ** 0.5).bfloat16()
    b = torch.randn(N, device=cuda).bfloat16()
    r = torch.randn(M, N, device=cuda).bfloat16()
    out = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
    ops.gemm_into(x, w, out, b, residual=r, force_cfg=SKINNY)
    want = x.float() @ w.float().t() + b.float() + r.float()
    assert _rel(out, want) < 1e-2


@pytest.mark.parametrize("act", ["silu", "gelu_tanh"])
def test_skinny_glu_and_act(cuda, act):
    M, N, K = 32, 2 * 2048, 4096
    x = torch.randn(M, K, device=cuda).bfloat16()
    w = (torch.randn(N, K, device=cuda) / K ** 0.5).bfloat16()
    out = torch.empty(M, N // 2, device=cuda, dtype=torch.bfloat16)
    ops.gemm_into(x, w, out, act=act, glu=True, force_cfg=SKINNY)
    y = x.float() @ w.float().t()
    f = torch.nn.functional.silu if act == "silu" else (lambda t: torch.nn.functional.gelu(t, approximate="tanh"))
    assert _rel(out, y[:, 0::2] * f(y[:, 1::2])) < 1e-2
    out2 = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
    ops.gemm_into(x, w, out2, act=act, force_cfg=SKINNY)
    assert _rel(out2, f(y)) < 1e-2


def test_skinny_graph_replay_rearms_tickets(cuda):
    """Split-K fixup tickets must re-arm so graph replays stay correct."""
    M, N, K = 8, 1024, 8192   # few tiles, long K -> several K groups
    x = torch.randn(M, K, device=cuda).bfloat16()
    w = (torch.randn(N, K, device=cuda) / K ** 0.5).bfloat16()
    out = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
    ops.gemm_into(x, w, out, force_cfg=SKINNY)  # eager first: allocates tickets
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ops.gemm_into(x, w, out, force_cfg=SKINNY)
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        ops.gemm_into(x, w, out, force_cfg=SKINNY)
    for i in range(5):
        x.copy_(torch.randn(M, K, device=cuda).bfloat16())
        g.replay()
        torch.cuda.synchronize()
        assert _rel(out, x.float() @ w.float().t()) < 1e-2, i


def test_autotuned_decode_shapes(cuda):
    """The tuner may pick skinny or a tile config; either way results are right."""
    for M, N, K in [(32, 6144, 4096), (32, 4096, 4096), (32, 28672, 4096), (32, 4096, 14336)]:
        x = torch.randn(M, K, device=cuda).bfloat16()
        w = (torch.randn(N, K, device=cuda) / K ** 0.5).bfloat16()
        y = ops.linear(x, w)
        assert _rel(y, x.float() @ w.float().t()) < 1e-2
