"""Attention modules on the fused flash-attention kernel.

Projections are fused (one GEMM for Q/K/V or K/V) and the attention kernel
reads Q/K/V as strided views of the fused projection output, so there is no
split/transpose copy between the GEMM and attention (the reference's
diffusers/transformers attention does head reshapes + transposes + sliced
softmax, app/run-sd.py:135).
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn

from .. import ops
from .layers import Linear


def merge_linear_keys(sd: dict, prefix: str, parts, merged: str, bias: bool = True) -> None:
    """In-place: sd[prefix+parts[i]+'.weight'] ... -> sd[prefix+merged+'.weight'] (row concat)."""
    wk = [prefix + p + ".weight" for p in parts]
    if all(k in sd for k in wk):
        sd[prefix + merged + ".weight"] = torch.cat([sd.pop(k) for k in wk], 0)
        bk = [prefix + p + ".bias" for p in parts]
        if bias and all(k in sd for k in bk):
            sd[prefix + merged + ".bias"] = torch.cat([sd.pop(k) for k in bk], 0)
        else:
            for k in bk:
                sd.pop(k, None)


class FusedSelfAttention(nn.Module):
    """Multi-head (optionally grouped-query) self-attention with a fused QKV GEMM."""

    def __init__(self, dim: int, heads: int, head_dim: Optional[int] = None, kv_heads: Optional[int] = None,
                 qkv_bias: bool = True, out_bias: bool = True, out_dim: Optional[int] = None):
        super().__init__()
        self.heads = heads
        self.kv_heads = kv_heads or heads
        self.head_dim = head_dim or dim // heads
        hd = self.head_dim
        self.qkv = Linear(dim, (self.heads + 2 * self.kv_heads) * hd, bias=qkv_bias)
        self.out = Linear(self.heads * hd, out_dim or dim, bias=out_bias)

    def split(self, qkv: torch.Tensor):
        B, T, _ = qkv.shape
        H, Hk, hd = self.heads, self.kv_heads, self.head_dim
        q = qkv[..., : H * hd].view(B, T, H, hd)
        k = qkv[..., H * hd:(H + Hk) * hd].view(B, T, Hk, hd)
        v = qkv[..., (H + Hk) * hd:].view(B, T, Hk, hd)
        return q, k, v

    def forward(self, x, residual=None, causal: bool = False, kv_lens=None, bias=None, scale=None):
        B, T, _ = x.shape
        q, k, v = self.split(self.qkv(x))
        o = ops.attention(q, k, v, scale=scale, causal=causal, kv_lens=kv_lens, bias=bias)
        return self.out(o.view(B, T, self.heads * self.head_dim), residual=residual)


class CrossAttention(nn.Module):
    """Q from x, fused K/V GEMM from the (static) context.  K/V can be precomputed
    once per request and reused for every denoising step."""

    def __init__(self, dim: int, ctx_dim: int, heads: int, head_dim: Optional[int] = None, qkv_bias: bool = False,
                 out_bias: bool = True):
        super().__init__()
        self.heads = heads
        self.head_dim = head_dim or dim // heads
        inner = heads * self.head_dim
        self.q = Linear(dim, inner, bias=qkv_bias)
        self.kv = Linear(ctx_dim, 2 * inner, bias=qkv_bias)
        self.out = Linear(inner, dim, bias=out_bias)

    def context_kv(self, ctx: torch.Tensor) -> torch.Tensor:
        return self.kv(ctx)

    def forward(self, x, ctx_kv: torch.Tensor, residual=None, kv_lens=None):
        B, T, _ = x.shape
        S = ctx_kv.shape[1]
        H, hd = self.heads, self.head_dim
        q = self.q(x).view(B, T, H, hd)
        k = ctx_kv[..., : H * hd].view(ctx_kv.shape[0], S, H, hd)
        v = ctx_kv[..., H * hd:].view(ctx_kv.shape[0], S, H, hd)
        o = ops.attention(q, k, v, kv_lens=kv_lens)
        return self.out(o.view(B, T, H * hd), residual=residual)
