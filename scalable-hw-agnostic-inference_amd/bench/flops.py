"""Analytic FLOP / byte accounting of a model forward by intercepting the op layer.

``count(fn)`` runs ``fn`` with ``shai_amd.ops`` GEMM/conv/attention replaced by
shape-only stand-ins (outputs are uninitialised tensors), so full-size models
can be costed on the CPU in seconds.  Used to turn rocprof kernel times into
achieved TFLOP/s (profiles/*.md).
"""
from __future__ import annotations

import contextlib
from collections import defaultdict

import torch

from .. import ops


class FlopCounter:
    def __init__(self):
        self.flops = defaultdict(float)
        self.calls = defaultdict(int)

    def add(self, kind, f):
        self.flops[kind] += f
        self.calls[kind] += 1

    @property
    def total(self):
        return sum(self.flops.values())

    def report(self):
        lines = [f"{k:12s} {v / 1e12:10.4f} TFLOP  ({self.calls[k]} calls)" for k, v in sorted(self.flops.items())]
        lines.append(f"{'total':12s} {self.total / 1e12:10.4f} TFLOP")
        return "\n".join(lines)


@contextlib.contextmanager
def count_flops():
    fc = FlopCounter()
    saved = {n: getattr(ops, n) for n in ("linear", "conv2d", "attention", "bmm", "groupnorm_stats", "layernorm",
                                          "groupnorm_apply", "bias_act", "softmax_")}

    def linear(x, w, bias=None, act=None, residual=None, glu=False, alpha=1.0, res_alpha=1.0):
        M = x.numel() // x.shape[-1]
        N, K = w.shape
        fc.add("linear", 2.0 * M * N * K)
        return torch.empty(*x.shape[:-1], N // 2 if glu else N, dtype=x.dtype, device=x.device)

    def conv2d(x, w, bias, kh, kw, stride=1, pad=0, upsample=False, x2=None, norm=None, temb=None, residual=None,
               act=None, res_alpha=1.0):
        N, H, W, _ = x.shape
        IH, IW = (2 * H, 2 * W) if upsample else (H, W)
        OH = (IH + 2 * pad - kh) // stride + 1
        OW = (IW + 2 * pad - kw) // stride + 1
        fc.add("conv", 2.0 * N * OH * OW * w.shape[0] * w.shape[1])
        return torch.empty(N, OH, OW, w.shape[0], dtype=x.dtype, device=x.device)

    def attention(q, k, v, scale=None, causal=False, causal_offset=0, kv_lens=None, q_lens=None, bias=None, out=None):
        B, Sq, H, D = q.shape
        Skv = k.shape[1]
        f = 4.0 * B * H * Sq * Skv * D
        fc.add("attention", f / 2 if causal else f)
        return torch.empty(q.shape, dtype=q.dtype, device=q.device)

    def bmm(a, w, alpha=1.0):
        B, M, K = a.shape
        fc.add("bmm", 2.0 * B * M * w.shape[-2] * K)
        return torch.empty(B, M, w.shape[-2], dtype=a.dtype, device=a.device)

    def gn_stats(x, gamma, beta, groups, eps, x2=None):
        N, C = x.shape[0], x.shape[-1] + (x2.shape[-1] if x2 is not None else 0)
        return torch.ones(N, C), torch.zeros(N, C)

    def gn_apply(x, scale, shift, silu=False, x2=None):
        return x if x2 is None else torch.empty(*x.shape[:-1], x.shape[-1] + x2.shape[-1], dtype=x.dtype)

    def ln(x, w, b, eps=1e-5, residual=None):
        return x, residual

    for n, f in (("linear", linear), ("conv2d", conv2d), ("attention", attention), ("bmm", bmm),
                 ("groupnorm_stats", gn_stats), ("layernorm", ln), ("groupnorm_apply", gn_apply),
                 ("bias_act", lambda x, *a, **k: x), ("softmax_", lambda x, *a, **k: x)):
        setattr(ops, n, f)
    try:
        yield fc
    finally:
        for n, f in saved.items():
            setattr(ops, n, f)


def sd21_unet_flops(batch: int = 2, res: int = 512) -> FlopCounter:
    """FLOPs of one SD2.1 UNet forward at `batch` (already CFG-doubled) and resolution."""
    from ..models import unet2d
    from ..models.unet2d import UNet2DConditionModel, UNetConfig
    unet = UNet2DConditionModel(UNetConfig.sd21())
    h = res // 8
    handoff = unet2d.NORM_HANDOFF
    unet2d.NORM_HANDOFF = False  # same GEMMs either way; the counter stubs the plain norm ops only
    try:
        with count_flops() as fc, torch.no_grad():
            ctx = torch.zeros(batch, 77, 1024, dtype=torch.bfloat16)
            kv = unet.context_kv(ctx)
            fc.flops.clear()
            fc.calls.clear()
            unet(torch.zeros(batch, h, h, 4, dtype=torch.bfloat16), torch.tensor([1.0]), kv)
    finally:
        unet2d.NORM_HANDOFF = handoff
    return fc


if __name__ == "__main__":
    print(sd21_unet_flops(2).report())
