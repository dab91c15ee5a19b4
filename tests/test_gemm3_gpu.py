"""Pipelined GEMM / conv kernels vs fp32 PyTorch (forced configs).

* gemm_8ph.hip (v4, 8-phase ping-pong): configs 9 (256x256) and 10 (256x320), 11 / 12 persistent.
* gemm_w4.hip (four-wave, one 128x128 wave tile per SIMD): config 13 (256x256) -- in production for the VAE
  decoder convs and the LLM prefill / Flux shapes, so every epilogue it implements is forced here too
  (test_w4_* below).
"""
import os
import subprocess
import sys

import pytest
import torch

from shai_amd import ops

pytestmark = pytest.mark.gpu
CFGS = [9, 10, 11, 12, 13]


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-6)).item()


@pytest.mark.parametrize("M,N,K", [(4096, 4096, 4096), (300, 520, 200), (1000, 256, 96), (257, 1024, 2048),
                                   (65536, 320, 320), (777, 650, 136), (70000, 700, 192)])
@pytest.mark.parametrize("cfg", CFGS)
def test_gemm3_plain_bias_residual(cuda, M, N, K, cfg):
    torch.manual_seed(M)
    a = torch.randn(M, K, device=cuda).bfloat16()
    w = (torch.randn(N, K, device=cuda) / K ** 0.5).bfloat16()
    bias = torch.randn(N, device=cuda).bfloat16()
    r = torch.randn(M, N, device=cuda).bfloat16()
    out = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
    ops.gemm_into(a, w, out, bias, residual=r, force_cfg=cfg)
    assert _rel(out, a.float() @ w.float().t() + bias.float() + r.float()) < 1e-2


@pytest.mark.parametrize("act", ["gelu", "silu"])
@pytest.mark.parametrize("cfg", CFGS)
def test_gemm3_glu(cuda, act, cfg):
    M, N, K = 2048, 2560, 320
    a = torch.randn(M, K, device=cuda).bfloat16()
    w = (torch.randn(N, K, device=cuda) / K ** 0.5).bfloat16()
    out = torch.empty(M, N // 2, device=cuda, dtype=torch.bfloat16)
    ops.gemm_into(a, w, out, act=act, glu=True, force_cfg=cfg)
    y = a.float() @ w.float().t()
    f = torch.nn.functional.gelu if act == "gelu" else torch.nn.functional.silu
    assert _rel(out, y[:, 0::2] * f(y[:, 1::2])) < 1e-2


@pytest.mark.parametrize("cfg", CFGS)
def test_gemm3_batched_strided(cuda, cfg):
    B, M, N, K = 3, 300, 384, 256
    a = torch.randn(B, M, K, device=cuda).bfloat16()
    w = torch.randn(N, K, device=cuda).bfloat16()
    j = torch.zeros(B, M + 40, N, device=cuda).bfloat16()
    ops.gemm_into(a, w, j[:, 40:], force_cfg=cfg)
    assert _rel(j[:, 40:], a.float() @ w.float().t()) < 1e-2 and j[:, :40].abs().sum().item() == 0


CONV_SCRIPT = r"""
import sys, torch
sys.path.insert(0, {root!r})
import shai_amd.ops as ops
from shai_amd.ops import reference as ref
torch.manual_seed(0)
cases = [(2, 32, 32, 64, 128, 3, 1, 1, False, 0), (2, 16, 16, 320, 320, 3, 1, 1, False, 0),
         (1, 16, 16, 64, 96, 3, 2, 1, False, 0), (2, 8, 8, 128, 64, 3, 1, 1, True, 0),
         (2, 16, 16, 96, 64, 3, 1, 1, False, 64), (2, 16, 16, 64, 64, 1, 1, 0, False, 0),
         (2, 32, 32, 320, 640, 3, 1, 1, False, 320), (2, 8, 8, 640, 320, 3, 1, 1, True, 640),
         (3, 12, 12, 128, 256, 3, 2, 1, False, 0),
         # > 256 output tiles: the persistent configs walk several tiles per workgroup
         (20, 64, 64, 320, 320, 3, 1, 1, False, 0), (8, 48, 48, 128, 256, 3, 1, 1, True, 0)]
worst = 0.0
for N, H, C, Co, k, stride, pad, up, c2 in [(c[0], c[1], c[3], c[4], c[5], c[6], c[7], c[8], c[9]) for c in cases]:
    x = torch.randn(N, H, H, C, device="cuda").bfloat16()
    x2 = torch.randn(N, H, H, c2, device="cuda").bfloat16() if c2 else None
    cin = C + c2
    w = (torch.randn(Co, cin, k, k, device="cuda") / (cin * k * k) ** 0.5).bfloat16()
    wp = ops.pack_conv_weight(w)
    b = torch.randn(Co, device="cuda").bfloat16()
    y = ops.conv2d(x, wp, b, k, k, stride, pad, upsample=up, x2=x2, act="silu")
    yr = ref.conv2d(x.cpu(), wp.cpu(), b.cpu(), k, k, stride, pad, upsample=up, x2=x2.cpu() if x2 is not None else None, act="silu")
    rel = ((y.float().cpu() - yr.float()).norm() / yr.float().norm()).item()
    worst = max(worst, rel)
print("WORST", worst)
assert worst < 2e-2, worst
"""


@pytest.mark.parametrize("cfg", CFGS)
def test_gemm3_conv_forced(cuda, cfg):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, SHAI_GEMM_FORCE=str(cfg))
    r = subprocess.run([sys.executable, "-c", CONV_SCRIPT.format(root=root)], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]


W4 = 13

UP2_SCRIPT = r"""
import math, sys, torch
sys.path.insert(0, {root!r})
import shai_amd.ops as ops
from shai_amd.ops import reference as ref
torch.manual_seed(5)
worst = 0.0
for (N, H, W, C, Co, act) in [(2, 16, 16, 1280, 1280, "silu"), (1, 32, 32, 640, 640, None), (4, 16, 32, 256, 512, None),
                              (8, 8, 8, 1280, 1280, None), (6, 8, 16, 256, 320, "silu")]:
    x = torch.randn(N, H, W, C, device="cuda").bfloat16()
    w = ops.pack_conv_weight((torch.randn(Co, C, 3, 3, device="cuda") / math.sqrt(C * 9)).bfloat16())
    b = torch.randn(Co, device="cuda").bfloat16()
    # image groups (H W < 256) take no per-image bias
    temb = torch.randn(N, Co, device="cuda").bfloat16() if H * W >= 256 else None
    assert ops.up2_phases_ok(x, 3, 3, 1, 1, temb=temb)
    y, gp = ops.conv2d(x, w, b, 3, 3, 1, 1, upsample=True, temb=temb, act=act, stats="gn",
                       w_up2=ops.pack_up2_phase_weight(w, C))
    yr = ref.conv2d(x, w, b, 3, 3, 1, 1, upsample=True, temb=temb, act=act)
    rel = ((y.float() - yr.float()).norm() / yr.float().norm()).item()
    worst = max(worst, rel)
    want = ref.col_partials(y.reshape(-1, Co)).reshape(N, -1, Co, 2).sum(1)
    torch.testing.assert_close(gp.reshape(N, -1, Co, 2).sum(1), want, atol=2e-1, rtol=1e-3)
print("WORST", worst)
assert worst < 1e-2, worst
"""


@pytest.mark.parametrize("cfg,splits", [(9, 1), (10, 1), (9, 3), (10, 4), (11, 1), (12, 2)])
def test_up2_phase_conv_forced(cuda, cfg, splits):
    """Phase-decomposed upsample conv on each v4 config, unsplit and split-K (the fold maps GEMM rows to output
    pixels), with per-image bias, SiLU and the output's GroupNorm partials (own process: SHAI_GEMM_FORCE /
    SHAI_GEMM_FORCE_SPLITS are read once per process)."""
    code = UP2_SCRIPT.format(root=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env = dict(os.environ, SHAI_GEMM_FORCE=str(cfg), SHAI_GEMM_FORCE_SPLITS=str(splits))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]


@pytest.mark.parametrize("act", ["gelu", "silu", "gelu_tanh"])
def test_w4_glu_acts_ragged(cuda, act):
    """GLU epilogue of the four-wave kernel with ragged M / N (edge tiles take the element-wise path)."""
    M, N, K = 777, 2 * 648, 320
    torch.manual_seed(1)
    a = torch.randn(M, K, device=cuda).bfloat16()
    w = (torch.randn(N, K, device=cuda) / K ** 0.5).bfloat16()
    b = torch.randn(N, device=cuda).bfloat16()
    out = torch.empty(M, N // 2, device=cuda, dtype=torch.bfloat16)
    ops.gemm_into(a, w, out, b, act=act, glu=True, force_cfg=W4)
    y = a.float() @ w.float().t() + b.float()
    f = {"gelu": torch.nn.functional.gelu, "silu": torch.nn.functional.silu,
         "gelu_tanh": lambda t: torch.nn.functional.gelu(t, approximate="tanh")}[act]
    assert _rel(out, y[:, 0::2] * f(y[:, 1::2])) < 1e-2


@pytest.mark.parametrize("M,N", [(512, 512), (600, 264)])
def test_w4_gate_residual_inplace(cuda, M, N):
    """out = x + gate[row // rpg] * act(x W^T + b), in place on the residual (AdaLN-Zero gated output)."""
    K, rpg = 384, 128
    torch.manual_seed(2)
    a = torch.randn(M, K, device=cuda).bfloat16()
    w = (torch.randn(N, K, device=cuda) / K ** 0.5).bfloat16()
    b = torch.randn(N, device=cuda).bfloat16()
    g = torch.randn((M + rpg - 1) // rpg, N, device=cuda).bfloat16()
    x = torch.randn(M, N, device=cuda).bfloat16()
    want = x.float() + g.float().repeat_interleave(rpg, 0)[:M] * torch.nn.functional.silu(a.float() @ w.float().t() + b.float())
    ops.gemm_into(a, w, x, b, act="silu", residual=x, gate=g, rows_per_gate=rpg, force_cfg=W4)
    assert _rel(x, want) < 1e-2


def test_w4_batched_alpha(cuda):
    """Batched strided operands (blockIdx.y) with alpha / res_alpha scaling."""
    B, M, N, K = 2, 520, 512, 256
    torch.manual_seed(3)
    a = torch.randn(B, M, K, device=cuda).bfloat16()
    w = torch.randn(N, K, device=cuda).bfloat16()
    r = torch.randn(B, M, N, device=cuda).bfloat16()
    j = torch.zeros(B, M + 8, N, device=cuda).bfloat16()
    ops.gemm_into(a, w, j[:, 8:], residual=r, alpha=0.5, res_alpha=-2.0, force_cfg=W4)
    assert _rel(j[:, 8:], 0.5 * (a.float() @ w.float().t()) - 2.0 * r.float()) < 1e-2
    assert j[:, :8].abs().sum().item() == 0


@pytest.mark.parametrize("up,c2", [(False, 0), (True, 0), (False, 256), (True, 128)])
def test_w4_conv_temb_residual(cuda, up, c2):
    """Implicit-GEMM conv on the four-wave kernel as the VAE decoder / UNet use it: nearest-2x upsample, channel
    concat, per-image bias (temb), SiLU, residual -- against the fp32 reference conv (own process: the forced
    config is read once per process from SHAI_GEMM_FORCE)."""
    code = CONV_W4_SCRIPT.format(root=os.path.dirname(os.path.dirname(os.path.abspath(__file__))), up=up, c2=c2)
    r = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, SHAI_GEMM_FORCE=str(W4)),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]


CONV_W4_SCRIPT = r"""
import sys, torch
sys.path.insert(0, {root!r})
import shai_amd.ops as ops
from shai_amd.ops import reference as ref
torch.manual_seed(4)
up, c2 = {up}, {c2}
N, H, C, Co = 2, 24, 256, 256
x = torch.randn(N, H, H, C, device="cuda").bfloat16()
x2 = torch.randn(N, H, H, c2, device="cuda").bfloat16() if c2 else None
cin = C + c2
w = (torch.randn(Co, cin, 3, 3, device="cuda") / (cin * 9) ** 0.5).bfloat16()
wp = ops.pack_conv_weight(w)
b = torch.randn(Co, device="cuda").bfloat16()
temb = torch.randn(N, Co, device="cuda").bfloat16()
OH = 2 * H if up else H
res = torch.randn(N, OH, OH, Co, device="cuda").bfloat16()
y = ops.conv2d(x, wp, b, 3, 3, 1, 1, upsample=up, x2=x2, temb=temb, residual=res, act="silu")
yr = ref.conv2d(x.cpu(), wp.cpu(), b.cpu(), 3, 3, 1, 1, upsample=up, x2=x2.cpu() if x2 is not None else None,
                temb=temb.cpu(), residual=res.cpu(), act="silu")
rel = ((y.float().cpu() - yr.float()).norm() / yr.float().norm()).item()
print("REL", rel)
assert rel < 2e-2, rel
"""


@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("splits", [1, 3])
@pytest.mark.parametrize("glu", [False, True])
def test_gemm2_every_tile_config_forced(cuda, cfg, splits, glu):
    """Every v2 tile config (gemm_lds.hip: 0 = 256x320, 1 = 256x256, 2 = 256x128, 3 = 128x128, 4 = 128x64 -- 0 and 1
    hold ~20 cached shapes with no other forced test) unsplit and split-K 3 (force 3000 + 100 splits + cfg), with
    bias + activation + residual (or the GLU epilogue), ragged M / N / K tails, against fp32."""
    torch.manual_seed(40 + cfg)
    M, N, K = 700, 1288 if not glu else 1280, 1000
    a = torch.randn(M, K, device=cuda).bfloat16()
    w = (torch.randn(N, K, device=cuda) / K ** 0.5).bfloat16()
    bias = torch.randn(N, device=cuda).bfloat16()
    No = N // 2 if glu else N
    r = torch.randn(M, No, device=cuda).bfloat16()
    out = torch.empty(M, No, device=cuda, dtype=torch.bfloat16)
    force = cfg if splits == 1 else 3000 + 100 * splits + cfg
    act = "gelu" if glu else "silu"
    ops.gemm_into(a, w, out, bias, act=act, residual=r, glu=glu, force_cfg=force)
    y = a.float() @ w.float().t() + bias.float()
    f = torch.nn.functional.gelu if glu else torch.nn.functional.silu
    want = (y[:, 0::2] * f(y[:, 1::2]) if glu else f(y)) + r.float()
    assert _rel(out, want) < 1e-2
