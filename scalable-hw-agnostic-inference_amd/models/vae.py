"""AutoencoderKL decoder (diffusers architecture), NHWC, shared by SD2.1 (4-ch
latents) and Flux.1 (16-ch latents, shift factor).

Reference: the VAE decode step of app/run-sd.py (diffusers) and the Neuron-traced
Flux decoder (app/src/decoder/model.py:6-18).  All convs are implicit-GEMM MFMA
with GroupNorm+SiLU fused into the gather and the residual fused into the
epilogue; the mid-block single-head attention (d=512) runs as two batched MFMA
GEMMs around a row-softmax kernel (head dim 512 exceeds the flash kernel's
register tile).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass
from typing import Tuple

import torch
import torch.nn as nn

from .. import ops
from .attention import merge_linear_keys
from .layers import Conv2d, GroupNorm, Linear
from .unet2d import ResnetBlock2D


@dataclass
class VAEConfig:
    latent_channels: int = 4
    out_channels: int = 3
    block_out_channels: Tuple[int, ...] = (128, 256, 512, 512)
    layers_per_block: int = 2
    norm_num_groups: int = 32
    scaling_factor: float = 0.18215
    shift_factor: float = 0.0
    use_post_quant_conv: bool = True

    @staticmethod
    def sd21():
        return VAEConfig()

    @staticmethod
    def flux():
        return VAEConfig(latent_channels=16, scaling_factor=0.3611, shift_factor=0.1159, use_post_quant_conv=False)

    @staticmethod
    def tiny(latent_channels=4):
        return VAEConfig(latent_channels=latent_channels, block_out_channels=(32, 32, 32, 64), layers_per_block=1)


# SHAI_VAE_FUSED_ATTN=0: the unfused score GEMM -> softmax -> value GEMM path (chunked scores)
VAE_FUSED_ATTN = os.environ.get("SHAI_VAE_FUSED_ATTN", "1") != "0"


class VAEAttention(nn.Module):
    SCORE_BYTES = 512 << 20

    def __init__(self, ch: int, groups: int):
        super().__init__()
        self.ch = ch
        self.group_norm = GroupNorm(groups, ch, 1e-6)
        self.qkv = Linear(ch, 3 * ch)
        self.out = Linear(ch, ch)

    def forward(self, x):
        B, H, W, C = x.shape
        h = self.group_norm(x).view(B, H * W, C)
        qkv = self.qkv(h)
        q, k, v = qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:]
        S = H * W
        if x.is_cuda and C in (64, 128, 512) and VAE_FUSED_ATTN:
            # fused flash attention on the strided q / k / v views of the qkv rows (one head; D = 512 is the
            # dedicated attention3.hip kernel): no S x S scores in HBM
            o = ops.attention(q.view(B, S, 1, C), k.view(B, S, 1, C), v.view(B, S, 1, C), scale=1.0 / math.sqrt(C))
            return self.out(o.view(B, S, C), residual=x.view(B, H * W, C)).view(B, H, W, C)
        k, vt = k.contiguous(), v.transpose(1, 2).contiguous()
        # single head, d = 512: score GEMM -> row softmax -> value GEMM, over query-row chunks so the bf16
        # score buffer stays <= SCORE_BYTES whatever the batch and resolution (768^2: S = 9216 -> 170 MB of
        # scores per image unchunked)
        rows = max(64, min(S, self.SCORE_BYTES // max(1, B * S * 2)) // 64 * 64)
        if rows >= S:
            s = ops.bmm(q.contiguous(), k, alpha=1.0 / math.sqrt(C))  # [B, S, S]
            ops.softmax_(s)
            o = ops.bmm(s, vt)  # [B, S, C]
        else:
            o = torch.empty(B, S, C, dtype=x.dtype, device=x.device)
            for r0 in range(0, S, rows):
                r1 = min(S, r0 + rows)
                s = ops.bmm(q[:, r0:r1].contiguous(), k, alpha=1.0 / math.sqrt(C))
                ops.softmax_(s)
                o[:, r0:r1] = ops.bmm(s, vt)
        return self.out(o, residual=x.view(B, H * W, C)).view(B, H, W, C)


class VAEMid(nn.Module):
    def __init__(self, ch, groups):
        super().__init__()
        self.resnets = nn.ModuleList([ResnetBlock2D(ch, ch, None, groups, 1e-6), ResnetBlock2D(ch, ch, None, groups, 1e-6)])
        self.attentions = nn.ModuleList([VAEAttention(ch, groups)])


class _Upsample(nn.Module):
    def __init__(self, ch):
        super().__init__()
        self.conv = Conv2d(ch, ch, 3, padding=1)


class VAEUpBlock(nn.Module):
    def __init__(self, cin, cout, n, groups, up):
        super().__init__()
        self.resnets = nn.ModuleList([ResnetBlock2D(cin if i == 0 else cout, cout, None, groups, 1e-6) for i in range(n)])
        self.upsamplers = nn.ModuleList([_Upsample(cout)]) if up else None


class Decoder(nn.Module):
    def __init__(self, cfg: VAEConfig):
        super().__init__()
        chs = list(reversed(cfg.block_out_channels))
        g = cfg.norm_num_groups
        self.conv_in = Conv2d(cfg.latent_channels, chs[0], 3, padding=1)
        self.mid_block = VAEMid(chs[0], g)
        self.up_blocks = nn.ModuleList()
        prev = chs[0]
        for i, c in enumerate(chs):
            self.up_blocks.append(VAEUpBlock(prev, c, cfg.layers_per_block + 1, g, i < len(chs) - 1))
            prev = c
        self.conv_norm_out = GroupNorm(g, chs[-1], 1e-6)
        self.conv_out = Conv2d(chs[-1], cfg.out_channels, 3, padding=1)

    def forward(self, z):
        x = self.conv_in(z)
        x = self.mid_block.resnets[0](x)
        x = self.mid_block.attentions[0](x)
        x = self.mid_block.resnets[1](x)
        for blk in self.up_blocks:
            for r in blk.resnets:
                x = r(x)
            if blk.upsamplers is not None:
                x = blk.upsamplers[0].conv(x, upsample=True)
        return self.conv_out(self.conv_norm_out(x, silu=True))


class AutoencoderKLDecoder(nn.Module):
    def __init__(self, cfg: VAEConfig = None):
        super().__init__()
        cfg = cfg or VAEConfig()
        self.cfg = cfg
        self.post_quant_conv = Conv2d(cfg.latent_channels, cfg.latent_channels, 1) if cfg.use_post_quant_conv else None
        self.decoder = Decoder(cfg)

    # Largest operand the tuned (v2/v3) GEMM/conv kernels address with 32-bit offsets; bigger operands fall
    # back to the register-staged v1 kernel (csrc/bindings.cpp use_v2), 2-4x slower on the full-res VAE convs.
    OPERAND_LIMIT = (1 << 31) - (1 << 24)

    def peak_bytes_per_image(self, h: int, w: int) -> int:
        """Largest bf16 activation (bytes) one image produces in the decoder, latent h x w."""
        rev = list(reversed(self.cfg.block_out_channels))
        f, peak, prev = 1, rev[0], rev[0]
        for i, c in enumerate(rev):
            peak = max(peak, f * f * max(prev, c))
            if i < len(rev) - 1:
                f *= 2
                peak = max(peak, f * f * c)
            prev = c
        return h * w * peak * 2

    def forward(self, latents: torch.Tensor) -> torch.Tensor:
        """latents NHWC [B, h, w, C] (scaled) -> image NHWC [B, 8h, 8w, 3] in [-1, 1].

        Large batches decode in balanced chunks whose activations stay under OPERAND_LIMIT, so every
        full-resolution conv runs on the tuned kernels (SD2.1 512^2: 11 images per chunk)."""
        B = latents.shape[0]
        per = max(1, self.OPERAND_LIMIT // self.peak_bytes_per_image(latents.shape[1], latents.shape[2]))
        if latents.is_cuda and B > per:
            n = -(-B // per)
            step = -(-B // n)
            return torch.cat([self._decode(latents[i:i + step]) for i in range(0, B, step)], 0)
        return self._decode(latents)

    def _decode(self, latents: torch.Tensor) -> torch.Tensor:
        lat = latents.contiguous()
        z = ops.bias_act(lat.view(-1, 8), None, None, None, alpha=1.0 / self.cfg.scaling_factor).view(lat.shape)
        if self.cfg.shift_factor:
            z = z + self.cfg.shift_factor
        if self.post_quant_conv is not None:
            z = self.post_quant_conv(z)
        return self.decoder(z)

    @staticmethod
    def to_uint8(img: torch.Tensor) -> torch.Tensor:
        return ((img.float() / 2 + 0.5).clamp(0, 1) * 255).round().to(torch.uint8)

    def convert_hf_state_dict(self, sd: dict) -> dict:
        out = {}
        for k, v in sd.items():
            if k.startswith("encoder.") or k.startswith("quant_conv."):
                continue
            k2 = k.replace(".to_out.0.", ".out.")
            if ".attentions." in k2 and v.dim() == 4:  # legacy 1x1-conv attention weights
                v = v[:, :, 0, 0]
            out[k2] = v
        for name, m in self.named_modules():
            if isinstance(m, VAEAttention):
                merge_linear_keys(out, name + ".", ["to_q", "to_k", "to_v"], "qkv")
        return out
