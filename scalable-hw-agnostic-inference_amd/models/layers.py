"""Building-block modules shared by every model family.

All activations are bf16 and channels-last (NHWC for images, [B, T, C] for
tokens).  Weights are stored in the layout the gfx950 kernels consume:

* ``Linear``: [out, in] (K-contiguous, the GEMM's "W" operand).
* ``GLULinear``: rows interleaved (value_i, gate_i) so SwiGLU/GEGLU is fused
  into the GEMM epilogue; HF checkpoints ([value; gate] halves, or separate
  gate/up projections) are interleaved at load time.
* ``Conv2d``: packed [out, KH*KW*Cin] (implicit-GEMM K order (kh, kw, c));
  HF [out, in, kh, kw] weights are repacked at load time.

``_load_from_state_dict`` hooks perform those conversions so HF/diffusers
safetensors load directly by parameter name (see ``shai_amd.weights``).
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn as nn

from .. import ops

BF16 = torch.bfloat16


def _round8(c: int) -> int:
    return (c + 7) // 8 * 8


class Linear(nn.Module):
    def __init__(self, in_features: int, out_features: int, bias: bool = True, dtype=BF16):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.weight = nn.Parameter(torch.empty(out_features, in_features, dtype=dtype), requires_grad=False)
        self.bias = nn.Parameter(torch.zeros(out_features, dtype=dtype), requires_grad=False) if bias else None

    def forward(self, x, act=None, residual=None, alpha: float = 1.0):
        return ops.linear(x, self.weight, self.bias, act=act, residual=residual, alpha=alpha)

    def forward_stats(self, x, residual=None, stats: str = "ln", eps: float = 1e-5):
        """(y, statistics of y for the next norm) -- see ``ops.linear_stats``."""
        return ops.linear_stats(x, self.weight, self.bias, residual=residual, stats=stats, eps=eps)

    def folded(self, ln: "LayerNorm"):
        """(w', bias', s) of this projection with LayerNorm ``ln`` folded in (``ops.fold_layernorm``); cached
        until the weights change."""
        return _folded(self, ln)


def _wkey(t):
    """Cache key of a derived weight: storage identity and version (inference-mode tensors carry no version counter:
    their storage identity is the key)."""
    return (t.data_ptr(), 0 if t.is_inference() else t._version) if t is not None else None


def _folded(lin, ln):
    key = tuple(_wkey(t) for t in (lin.weight, lin.bias, ln.weight, ln.bias))
    cache = getattr(lin, "_ln_fold", None)
    if cache is None or cache[0] != key:
        cache = (key, ops.fold_layernorm(lin.weight, lin.bias, ln.weight, ln.bias))
        lin._ln_fold = cache
    return cache[1]


class GLULinear(nn.Module):
    """Linear producing 2*F features consumed as value * act(gate) -> F outputs.

    ``hf_layout='halves'``: checkpoint weight is [value; gate] (diffusers GEGLU).
    """

    def __init__(self, in_features: int, hidden: int, bias: bool = True, act: str = "gelu", dtype=BF16,
                 hf_layout: str = "halves"):
        super().__init__()
        self.in_features, self.hidden, self.act, self.hf_layout = in_features, hidden, act, hf_layout
        self.weight = nn.Parameter(torch.empty(2 * hidden, in_features, dtype=dtype), requires_grad=False)
        self.bias = nn.Parameter(torch.zeros(2 * hidden, dtype=dtype), requires_grad=False) if bias else None

    @staticmethod
    def interleave(value: torch.Tensor, gate: torch.Tensor) -> torch.Tensor:
        return torch.stack([value, gate], dim=1).reshape(-1, *value.shape[1:])

    def _load_from_state_dict(self, state_dict, prefix, *args, **kwargs):
        for name in ("weight", "bias"):
            k = prefix + name
            if k in state_dict and not getattr(state_dict[k], "_shai_interleaved", False):
                t = state_dict[k]
                h = t.shape[0] // 2
                t2 = self.interleave(t[:h], t[h:])
                t2._shai_interleaved = True
                state_dict[k] = t2
        super()._load_from_state_dict(state_dict, prefix, *args, **kwargs)

    def forward(self, x, residual=None):
        return ops.linear(x, self.weight, self.bias, act=self.act, residual=residual, glu=True)

    def folded(self, ln: "LayerNorm"):
        return _folded(self, ln)


class Conv2d(nn.Module):
    """NHWC conv on the implicit-GEMM kernel. Input channels padded to a multiple of 8."""

    def __init__(self, cin: int, cout: int, kernel: int, stride: int = 1, padding: int = 0, bias: bool = True,
                 dtype=BF16):
        super().__init__()
        self.cin, self.cout, self.k, self.stride, self.padding = cin, cout, kernel, stride, padding
        self.cin_p = _round8(cin)
        self.weight = nn.Parameter(torch.empty(cout, kernel * kernel * self.cin_p, dtype=dtype), requires_grad=False)
        self.bias = nn.Parameter(torch.zeros(cout, dtype=dtype), requires_grad=False) if bias else None

    def pack(self, w4: torch.Tensor) -> torch.Tensor:
        if w4.shape[1] != self.cin_p:
            w4 = torch.nn.functional.pad(w4, (0, 0, 0, 0, 0, self.cin_p - w4.shape[1]))
        return ops.pack_conv_weight(w4)

    def _load_from_state_dict(self, state_dict, prefix, *args, **kwargs):
        k = prefix + "weight"
        if k in state_dict and state_dict[k].dim() == 4:
            state_dict[k] = self.pack(state_dict[k])
        super()._load_from_state_dict(state_dict, prefix, *args, **kwargs)

    def _phase_weight(self) -> torch.Tensor:
        """Phase weights of the upsample conv (ops.pack_up2_phase_weight), rebuilt when the weight changes."""
        key = _wkey(self.weight)
        cached = getattr(self, "_w_up2", None)
        if cached is None or cached[0] != key:
            if torch.cuda.is_current_stream_capturing():  # never first-built inside a graph capture: plain path
                return None
            cached = (key, ops.pack_up2_phase_weight(self.weight.data, self.cin_p))
            self._w_up2 = cached
        return cached[1]

    def _pad_in(self, x):
        if x.shape[-1] != self.cin_p:
            x = torch.nn.functional.pad(x, (0, self.cin_p - x.shape[-1]))
        return x

    def forward(self, x, norm=None, temb=None, residual=None, upsample: bool = False, x2=None, act=None,
                stats=None, eps: float = 1e-5):
        """stats="gn" / "ln": returns (out, statistics of out for the next norm), see ``ops.conv2d``."""
        if x2 is None:
            x = self._pad_in(x)
        extra = {} if stats is None else {"stats": stats, "eps": eps}
        if upsample and ops.up2_phases_ok(x, self.k, self.k, self.stride, self.padding, x2, norm, residual, self.cout,
                                          temb):
            w_up2 = self._phase_weight()
            if w_up2 is not None:
                extra["w_up2"] = w_up2
        return ops.conv2d(x, self.weight, self.bias, self.k, self.k, self.stride, self.padding, upsample=upsample,
                          x2=x2, norm=norm, temb=temb, residual=residual, act=act, **extra)


class GroupNorm(nn.Module):
    def __init__(self, groups: int, channels: int, eps: float = 1e-5, dtype=BF16):
        super().__init__()
        self.groups, self.channels, self.eps = groups, channels, eps
        self.weight = nn.Parameter(torch.ones(channels, dtype=dtype), requires_grad=False)
        self.bias = nn.Parameter(torch.zeros(channels, dtype=dtype), requires_grad=False)

    def stats(self, x, x2=None):
        """(scale, shift) fp32 [N, C]: fed to a consumer conv's fused prologue."""
        return ops.groupnorm_stats(x, self.weight, self.bias, self.groups, self.eps, x2=x2)

    def scale_shift(self, x, x2=None, part=None, part2=None):
        """(scale, shift) fp32 [N, C] of GroupNorm(cat([x, x2], -1)), from the producers' partials when given --
        the ``norm=`` prologue of a consumer conv (``ops.conv2d``)."""
        if part is not None and (x2 is None or part2 is not None):
            return ops.groupnorm_stats_from_partials(part, self.weight, self.bias, self.groups, self.eps, x.shape[0],
                                                     x.numel() // (x.shape[0] * x.shape[-1]),
                                                     part2=part2 if x2 is not None else None)
        return self.stats(x, x2)

    def forward(self, x, silu: bool = False, x2=None, part=None, part2=None):
        """GroupNorm of x, or of cat([x, x2], -1) without materialising the concat.  ``part`` / ``part2``:
        partials of x / x2 handed over by their producing GEMM (``conv2d(stats="gn")``), which replace the
        statistics pass over the input."""
        sc, sh = self.scale_shift(x, x2, part, part2)
        return ops.groupnorm_apply(x, sc, sh, silu, x2=x2)


class LayerNorm(nn.Module):
    def __init__(self, dim: int, eps: float = 1e-5, affine: bool = True, bias: bool = True, dtype=BF16):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(dim, dtype=dtype), requires_grad=False) if affine else None
        self.bias = nn.Parameter(torch.zeros(dim, dtype=dtype), requires_grad=False) if (affine and bias) else None

    def forward(self, x, residual=None):
        y, r = ops.layernorm(x, self.weight, self.bias, self.eps, residual)
        return (y, r) if residual is not None else y


class RMSNorm(nn.Module):
    def __init__(self, dim: int, eps: float = 1e-6, dtype=BF16, w_offset: float = 0.0):
        super().__init__()
        self.eps, self.w_offset = eps, w_offset
        self.weight = nn.Parameter(torch.ones(dim, dtype=dtype), requires_grad=False)

    def forward(self, x, residual=None):
        y, r = ops.rmsnorm(x, self.weight, self.eps, residual, self.w_offset)
        return (y, r) if residual is not None else y


class Embedding(nn.Module):
    def __init__(self, num: int, dim: int, dtype=BF16):
        super().__init__()
        self.weight = nn.Parameter(torch.empty(num, dim, dtype=dtype), requires_grad=False)

    def forward(self, ids):
        return ops.embedding(ids, self.weight)


def timestep_embedding(t: torch.Tensor, dim: int, flip_sin_to_cos: bool = True, shift: float = 0.0,
                       max_period: float = 10000.0, scale: float = 1.0) -> torch.Tensor:
    """Sinusoidal timestep features [B, dim] in fp32 (diffusers get_timestep_embedding semantics)."""
    half = dim // 2
    exponent = -math.log(max_period) * torch.arange(half, dtype=torch.float32, device=t.device) / (half - shift)
    emb = t.float()[:, None] * torch.exp(exponent)[None, :] * scale
    emb = torch.cat([torch.sin(emb), torch.cos(emb)], dim=-1)
    if flip_sin_to_cos:
        emb = torch.cat([emb[:, half:], emb[:, :half]], dim=-1)
    return emb


@torch.no_grad()
def init_random_(module: nn.Module, seed: int = 0, std_scale: float = 1.0) -> nn.Module:
    """Deterministic random init of a model (no checkpoints on the offline GPU box).

    Linear/Conv weights ~ N(0, 1/fan_in), norms identity, embeddings N(0, 0.02).
    Generated directly on the module's device.
    """
    covered = set()
    for i, (name, m) in enumerate(module.named_modules()):
        own = list(m.parameters(recurse=False))
        if not own:
            continue
        g = torch.Generator(device=own[0].device)
        g.manual_seed(seed * 1000003 + i)
        if hasattr(m, "full_shape") and hasattr(m, "_shard"):
            # tensor-parallel layer: draw the FULL (unsharded) tensor from the shared seed and keep this rank's
            # shard, so a TP=n replica holds exactly the TP=1 model's weights (random-init serving at any TP)
            for pname, p in m._parameters.items():
                if p is None:
                    continue
                full = m.full_shape(pname)
                if pname == "weight" and len(full) == 2 and not hasattr(m, "vocab"):
                    std = std_scale / math.sqrt(full[1])
                else:
                    std = 0.02
                t = torch.randn(full, generator=g, device=p.device) * std
                p.copy_(m._shard(pname, t) if tuple(full) != tuple(p.shape) else t)
                covered.add(id(p))
            continue
        if isinstance(m, (Linear, GLULinear, Conv2d, Embedding, GroupNorm, LayerNorm, RMSNorm)):
            covered.update(id(p) for p in own)
        else:
            for p in own:
                if id(p) not in covered:
                    p.copy_(torch.randn(p.shape, generator=g, device=p.device) * 0.02)
                    covered.add(id(p))
        if isinstance(m, (Linear, GLULinear)):
            fan = m.weight.shape[1]
            m.weight.copy_(torch.randn(m.weight.shape, generator=g, device=m.weight.device) * (std_scale / math.sqrt(fan)))
            if m.bias is not None:
                m.bias.copy_(torch.randn(m.bias.shape, generator=g, device=m.bias.device) * 0.02)
        elif isinstance(m, Conv2d):
            fan = m.k * m.k * m.cin
            w = torch.randn(m.cout, m.cin, m.k, m.k, generator=g, device=m.weight.device) * (std_scale / math.sqrt(fan))
            m.weight.copy_(m.pack(w))
            if m.bias is not None:
                m.bias.copy_(torch.randn(m.bias.shape, generator=g, device=m.bias.device) * 0.02)
        elif isinstance(m, Embedding):
            m.weight.copy_(torch.randn(m.weight.shape, generator=g, device=m.weight.device) * 0.02)
        elif isinstance(m, (GroupNorm, LayerNorm, RMSNorm)):
            if m.weight is not None:
                m.weight.fill_(1.0)
            if getattr(m, "bias", None) is not None:
                m.bias.zero_()
    return module
