"""Llama-3.2-Vision (mllama): tiled ViT-H/14 vision tower + Llama-3.1 text decoder with
gated cross-attention layers.

The reference serves it through vLLM-neuron at TP32 behind the multimodal
``/generate`` API (app/vllm_model_api_m.py:42-66 ``multi_modal_data={"image": ...}``,
cova/mllama-32-11b-vllm-trn1-config.yaml:7-23) and uses it as the caption stage of
the cova chain (app/cova_gradio_m.py:53-60).  Here it runs on the native LLM
engine (paged KV, continuous batching, HIP-graph decode):

* Vision tower: up to 4 tiles of 560x560 (14x14 patches, 1601 tokens/tile incl.
  CLS, padded to 1608), 32 local + 8 tanh-gated global pre-LN layers over ALL
  tiles at once, gated tile / aspect-ratio position embeddings, 5 intermediate
  layer outputs concatenated to the final state (7680 features), projected to the
  text width.  GEMMs on the MFMA GEMM kernel, attention on the flash kernel (the
  80-wide heads are zero-padded to 128 on the GPU; the scale stays 1/sqrt(80)).
  The aspect-ratio mask semantics of the original (valid queries see every key,
  padding queries see only valid keys) are kept exactly: the padding rows are
  recomputed against the gathered valid keys.
* Cross-attention K/V of the image are computed ONCE at prefill (k_norm applied)
  and written into the paged cache slab of each cross layer under a separate
  per-sequence block list; decode reuses them through the paged decode kernel.
  All tanh gates are folded into the weights of the GEMM that produces the gated
  branch (o_proj / down_proj / fc2), the norm gains into q_proj / gate_up (RMS
  scaling fused into the GEMM like the self-attention layers).
* Text rows before the ``<|image|>`` token follow the original
  full_text_row_masked_out semantics (attend to every tile, MLP branch zeroed);
  text-only batches skip the cross layers.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn as nn

from .. import ops
from ..parallel.layers import (ColumnParallelLinear, ParallelLMHead, QKVParallelLinear, RowParallelLinear,
                               VocabParallelEmbedding)
from .attention import merge_linear_keys
from .layers import Conv2d, GLULinear, LayerNorm, Linear, RMSNorm
from .llama import Batch, LlamaConfig, LlamaDecoderLayer, LlamaForCausalLM, LlamaMLP

CLIP_MEAN = (0.48145466, 0.4578275, 0.40821073)
CLIP_STD = (0.26862954, 0.26130258, 0.27577711)


def supported_aspect_ratios(max_tiles: int) -> List[Tuple[int, int]]:
    return [(a, b) for a in range(1, max_tiles + 1) for b in range(1, max_tiles + 1) if a * b <= max_tiles]


@dataclass
class MllamaVisionConfig:
    hidden_size: int = 1280
    num_hidden_layers: int = 32
    num_global_layers: int = 8
    attention_heads: int = 16
    intermediate_size: int = 5120
    vision_output_dim: int = 7680
    image_size: int = 560
    patch_size: int = 14
    norm_eps: float = 1e-5
    max_num_tiles: int = 4
    intermediate_layers_indices: Tuple[int, ...] = (3, 7, 15, 23, 30)
    image_mean: Tuple[float, ...] = CLIP_MEAN
    image_std: Tuple[float, ...] = CLIP_STD

    @property
    def num_patches(self) -> int:
        return (self.image_size // self.patch_size) ** 2 + 1

    @property
    def padded_patches(self) -> int:
        return (self.num_patches + 7) // 8 * 8

    @property
    def max_aspect_ratio_id(self) -> int:
        return len(supported_aspect_ratios(self.max_num_tiles))


def _llama32_text() -> LlamaConfig:
    return LlamaConfig(vocab_size=128256, hidden_size=4096, intermediate_size=14336, num_hidden_layers=40,
                       num_attention_heads=32, num_key_value_heads=8, head_dim=128, rope_theta=5e5,
                       max_position_embeddings=131072, bos_token_id=128000, eos_token_id=128009,
                       rope_scaling={"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0,
                                     "high_freq_factor": 4.0, "original_max_position_embeddings": 8192})


@dataclass
class MllamaConfig:
    text: LlamaConfig = field(default_factory=_llama32_text)
    vision: MllamaVisionConfig = field(default_factory=MllamaVisionConfig)
    cross_attention_layers: Tuple[int, ...] = (3, 8, 13, 18, 23, 28, 33, 38)
    image_token_index: int = 128256

    @staticmethod
    def llama32_11b_vision():
        return MllamaConfig()

    @staticmethod
    def tiny():
        text = LlamaConfig(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=4,
                           num_attention_heads=4, num_key_value_heads=2, head_dim=64, rope_theta=5e5,
                           max_position_embeddings=2048, bos_token_id=1, eos_token_id=2)
        vis = MllamaVisionConfig(hidden_size=64, num_hidden_layers=4, num_global_layers=2, attention_heads=2,
                                 intermediate_size=128, vision_output_dim=64 * 3, image_size=56, patch_size=14,
                                 max_num_tiles=4, intermediate_layers_indices=(1, 3))
        return MllamaConfig(text=text, vision=vis, cross_attention_layers=(1, 3), image_token_index=512)

    @staticmethod
    def from_hf(d: dict) -> "MllamaConfig":
        t, v = dict(d["text_config"]), d["vision_config"]
        rp = t.get("rope_parameters") or {}
        if "rope_theta" in rp:
            t["rope_theta"] = rp["rope_theta"]
        t["rope_scaling"] = t.get("rope_scaling") or (rp if rp.get("rope_type", "default") != "default" else None)
        text = LlamaConfig.from_hf(t)
        vis = MllamaVisionConfig(hidden_size=v["hidden_size"], num_hidden_layers=v["num_hidden_layers"],
                                 num_global_layers=v["num_global_layers"], attention_heads=v["attention_heads"],
                                 intermediate_size=v["intermediate_size"], vision_output_dim=v["vision_output_dim"],
                                 image_size=v["image_size"], patch_size=v["patch_size"],
                                 norm_eps=v.get("norm_eps", 1e-5), max_num_tiles=v["max_num_tiles"],
                                 intermediate_layers_indices=tuple(v["intermediate_layers_indices"]))
        return MllamaConfig(text=text, vision=vis, cross_attention_layers=tuple(t["cross_attention_layers"]),
                            image_token_index=d.get("image_token_index", 128256))


# ----------------------------------------------------------------------------- image preprocessing
def _optimal_canvas(h: int, w: int, max_tiles: int, tile: int) -> Tuple[int, int]:
    """(canvas_h, canvas_w) of the tile arrangement needing the smallest upscale (else the mildest
    downscale), ties broken by area -- the Llama-3.2-Vision processor's canvas rule."""
    arr = np.array(supported_aspect_ratios(max_tiles)) * tile
    th, tw = arr.T
    scales = np.minimum(th / h, tw / w)
    up = scales[scales >= 1]
    sel = up.min() if len(up) else scales[scales < 1].max()
    cand = arr[scales == sel]
    best = cand[np.argmin(cand[:, 0] * cand[:, 1])] if len(cand) > 1 else cand[0]
    return int(best[0]), int(best[1])


def _fit_to_canvas(h: int, w: int, ch: int, cw: int, tile: int) -> Tuple[int, int]:
    tw = int(np.clip(w, tile, cw))
    th = int(np.clip(h, tile, ch))
    sh, sw = th / h, tw / w
    if sw < sh:
        return min(math.floor(h * sw) or 1, th), tw
    return th, min(math.floor(w * sh) or 1, tw)


def preprocess_image(image, vcfg: MllamaVisionConfig, device="cpu") -> dict:
    """PIL image / HWC uint8 array -> {"pixel_values": [max_tiles, S, S, 3] bf16 NHWC (normalised; tiles past
    the valid ones are zero), "aspect_ratio_id": int, "num_tiles": int}.  Resize (bilinear, aspect preserved)
    to the optimal tiled canvas, pad bottom/right with black, normalise, split row-major into tiles."""
    from PIL import Image
    if isinstance(image, np.ndarray):
        image = Image.fromarray(image)
    image = image.convert("RGB")
    tile = vcfg.image_size
    w0, h0 = image.size
    ch, cw = _optimal_canvas(h0, w0, vcfg.max_num_tiles, tile)
    nh, nw = _fit_to_canvas(h0, w0, ch, cw, tile)
    img = np.asarray(image.resize((nw, nh), Image.BILINEAR), dtype=np.float32) / 255.0
    canvas = np.zeros((ch, cw, 3), np.float32)
    canvas[:nh, :nw] = img
    canvas = (canvas - np.asarray(vcfg.image_mean, np.float32)) / np.asarray(vcfg.image_std, np.float32)
    rows, cols = ch // tile, cw // tile
    tiles = canvas.reshape(rows, tile, cols, tile, 3).transpose(0, 2, 1, 3, 4).reshape(rows * cols, tile, tile, 3)
    px = np.zeros((vcfg.max_num_tiles, tile, tile, 3), np.float32)
    px[:rows * cols] = tiles
    ar_id = supported_aspect_ratios(vcfg.max_num_tiles).index((rows, cols)) + 1
    return {"pixel_values": torch.from_numpy(px).to(device=device, dtype=torch.bfloat16),
            "aspect_ratio_id": ar_id, "num_tiles": rows * cols}


# ----------------------------------------------------------------------------- vision tower
def _attn_any_head_dim(q, k, v, scale):
    """Flash attention for head dims the kernel does not tile (80): zero-pad to 128 on the GPU."""
    D = q.shape[-1]
    if not q.is_cuda or D in (64, 128):
        return ops.attention(q, k, v, scale=scale)
    Dp = 64 if D < 64 else 128
    pad = lambda t: torch.nn.functional.pad(t, (0, Dp - D))
    return ops.attention(pad(q), pad(k), pad(v), scale=scale)[..., :D]


class VisionAttention(nn.Module):
    """Head-sharded at TP > 1 (the reference serves the whole model under vLLM TP32,
    cova/mllama-32-11b-vllm-trn1-config.yaml:9; here the vision tower's 16 heads shard over TP <= 16): fused QKV
    column-parallel by heads, o_proj row-parallel with the residual added after the reduction -- each rank runs
    attention for its own heads over all tiles."""

    def __init__(self, c: MllamaVisionConfig):
        super().__init__()
        self.hd = c.hidden_size // c.attention_heads
        self.qkv = QKVParallelLinear(c.hidden_size, c.attention_heads, c.attention_heads, self.hd, bias=False)
        self.h = self.qkv.h_local
        self.o_proj = RowParallelLinear(c.hidden_size, c.hidden_size, bias=False)

    def forward(self, x, valid_idx: List[torch.Tensor], pad_idx: List[Optional[torch.Tensor]], residual):
        N, T, d = x.shape
        h, hd = self.h, self.hd
        dl = h * hd                      # this rank's heads
        qkv = self.qkv(x)
        q = qkv[..., :dl].view(N, T, h, hd)
        k = qkv[..., dl:2 * dl].view(N, T, h, hd)
        v = qkv[..., 2 * dl:].view(N, T, h, hd)
        scale = hd ** -0.5
        o = _attn_any_head_dim(q, k, v, scale).contiguous()
        for n in range(N):
            if pad_idx[n] is None:
                continue
            # padding queries see only valid keys (the original additive mask is -inf on pad x pad)
            pi, vi = pad_idx[n], valid_idx[n]
            op = _attn_any_head_dim(q[n:n + 1].index_select(1, pi), k[n:n + 1].index_select(1, vi),
                                    v[n:n + 1].index_select(1, vi), scale)
            o[n].index_copy_(0, pi, op[0])
        return self.o_proj(o.view(N, T, dl), residual=residual)


class VisionLayer(nn.Module):
    def __init__(self, c: MllamaVisionConfig, gated: bool):
        super().__init__()
        self.gated = gated
        self.input_layernorm = LayerNorm(c.hidden_size, c.norm_eps)
        self.self_attn = VisionAttention(c)
        self.post_attention_layernorm = LayerNorm(c.hidden_size, c.norm_eps)
        self.fc1 = ColumnParallelLinear(c.hidden_size, c.intermediate_size)      # MLP sharded by the hidden dim
        self.fc2 = RowParallelLinear(c.intermediate_size, c.hidden_size)
        if gated:
            self.gate_attn = nn.Parameter(torch.zeros(1), requires_grad=False)
            self.gate_ffn = nn.Parameter(torch.zeros(1), requires_grad=False)
        self._gates_folded = False

    @torch.no_grad()
    def fold_gates(self):
        """tanh(g) * (x W^T + b) == x (tanh(g) W)^T + tanh(g) b: scale the producing GEMM's weights once."""
        if not self.gated or self._gates_folded:
            return
        ga, gf = torch.tanh(self.gate_attn.float()), torch.tanh(self.gate_ffn.float())
        w = self.self_attn.o_proj.weight
        w.copy_((w.float() * ga).to(w.dtype))
        for p in (self.fc2.weight, self.fc2.bias):
            p.copy_((p.float() * gf).to(p.dtype))
        # tanh(inf) == 1: a folded state dict re-loaded into another model folds as a no-op
        self.gate_attn.fill_(float("inf"))
        self.gate_ffn.fill_(float("inf"))
        self._gates_folded = True

    def forward(self, x, valid_idx, pad_idx):
        x = self.self_attn(self.input_layernorm(x), valid_idx, pad_idx, residual=x)
        return self.fc2(self.fc1(self.post_attention_layernorm(x), act="gelu"), residual=x)


class MllamaVisionModel(nn.Module):
    # ``quantization: fp8`` quantises the language model only: the vision tower's prefill-sized GEMMs stay bf16
    # (parallel.layers.quantize_fp8_ skips every linear under a ``no_fp8`` module)
    no_fp8 = True

    def __init__(self, c: MllamaVisionConfig):
        super().__init__()
        self.cfg = c
        d, T, P = c.hidden_size, c.max_num_tiles, c.num_patches
        bf = torch.bfloat16
        self.patch_embedding = Conv2d(3, d, c.patch_size, stride=c.patch_size, bias=False)
        self.class_embedding = nn.Parameter(torch.empty(d, dtype=bf), requires_grad=False)
        self.pos_embedding = nn.Parameter(torch.empty(P, d, dtype=bf), requires_grad=False)
        self.pos_gate = nn.Parameter(torch.zeros(1), requires_grad=False)
        self.tile_pos_embedding = nn.Parameter(torch.empty(c.max_aspect_ratio_id + 1, T * P * d, dtype=bf),
                                               requires_grad=False)
        self.pre_tile_embedding = nn.Parameter(torch.empty(c.max_aspect_ratio_id + 1, T * d, dtype=bf),
                                               requires_grad=False)
        self.pre_tile_gate = nn.Parameter(torch.zeros(1), requires_grad=False)
        self.post_tile_embedding = nn.Parameter(torch.empty(c.max_aspect_ratio_id + 1, T * d, dtype=bf),
                                                requires_grad=False)
        self.post_tile_gate = nn.Parameter(torch.zeros(1), requires_grad=False)
        self.layernorm_pre = LayerNorm(d, 1e-5)
        self.layernorm_post = LayerNorm(d, 1e-5)
        self.layers = nn.ModuleList([VisionLayer(c, False) for _ in range(c.num_hidden_layers)])
        self.global_layers = nn.ModuleList([VisionLayer(c, True) for _ in range(c.num_global_layers)])

    def _indices(self, n_tiles: Sequence[int], device):
        """Per image: (valid token indices, padding token indices or None) of the [tiles * padded_patches] rows."""
        c = self.cfg
        P, Pp, T = c.num_patches, c.padded_patches, c.max_num_tiles
        valid, pad = [], []
        for nt in n_tiles:
            m = np.zeros((T, Pp), bool)
            m[:max(1, int(nt)), :P] = True
            m = m.reshape(-1)
            valid.append(torch.from_numpy(np.nonzero(m)[0]).to(device))
            pi = np.nonzero(~m)[0]
            pad.append(torch.from_numpy(pi).to(device) if len(pi) else None)
        return valid, pad

    def forward(self, pixel_values: torch.Tensor, aspect_ratio_ids: torch.Tensor, num_tiles: Sequence[int]):
        """pixel_values [N, T, S, S, 3] bf16 NHWC -> [N, T * P, vision_output_dim]."""
        c = self.cfg
        N, T, S = pixel_values.shape[:3]
        d, P, Pp = c.hidden_size, c.num_patches, c.padded_patches
        g = S // c.patch_size
        ar = aspect_ratio_ids.long().view(N)
        for layer in self.global_layers:
            layer.fold_gates()
        x = self.patch_embedding(pixel_values.reshape(N * T, S, S, 3)).view(N, T, g * g, d).float()
        x = x + self.pre_tile_embedding[ar].view(N, T, 1, d).float() * torch.tanh(self.pre_tile_gate.float())
        cls = self.class_embedding.float().view(1, 1, 1, d).expand(N, T, 1, d)
        x = torch.cat([cls, x], dim=2)                                   # [N, T, P, d]
        gp = torch.tanh(self.pos_gate.float())
        x = x + (1 - gp) * self.pos_embedding.float().view(1, 1, P, d)
        x = x + gp * self.tile_pos_embedding[ar].view(N, T, P, d).float()
        x = self.layernorm_pre(x.to(torch.bfloat16))
        x = torch.nn.functional.pad(x, (0, 0, 0, Pp - P)).reshape(N, T * Pp, d).contiguous()
        valid, pad = self._indices(num_tiles, x.device)
        inter = []
        want = set(c.intermediate_layers_indices)
        for i, layer in enumerate(self.layers):
            x = layer(x, valid, pad)
            if i in want:
                inter.append(x)
        x = self.layernorm_post(x)
        post = self.post_tile_embedding[ar].view(N, T, 1, d).float() * torch.tanh(self.post_tile_gate.float())
        x = (x.view(N, T, Pp, d).float() + post).to(torch.bfloat16).view(N, T * Pp, d).contiguous()
        for layer in self.global_layers:
            x = layer(x, valid, pad)
        x = x.view(N, T, Pp, d)[:, :, :P]
        st = torch.stack(inter, dim=-1).view(N, T, Pp, -1)[:, :, :P]   # channel-major, layer-minor (as HF)
        return torch.cat([x, st], dim=-1).reshape(N, T * P, -1).contiguous()


# ----------------------------------------------------------------------------- text decoder
class CrossAttention(nn.Module):
    """Cross-attention to the image K/V held in the paged cache (TP: heads sharded)."""

    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.q_proj = ColumnParallelLinear(cfg.hidden_size, cfg.num_attention_heads * cfg.head_dim, bias=False)
        self.kv_proj = QKVParallelLinear(cfg.hidden_size, 0, cfg.num_key_value_heads, cfg.head_dim)
        self.o_proj = RowParallelLinear(cfg.num_attention_heads * cfg.head_dim, cfg.hidden_size, bias=False)
        self.q_norm = RMSNorm(cfg.head_dim, cfg.rms_norm_eps)
        self.k_norm = RMSNorm(cfg.head_dim, cfg.rms_norm_eps)
        self.h = self.q_proj.out_local // cfg.head_dim
        self.hk = self.kv_proj.kv_local
        self.hd = cfg.head_dim
        self.scale = cfg.head_dim ** -0.5

    def write_image_kv(self, states: torch.Tensor, k_cache, v_cache, slots: torch.Tensor):
        """states [Nv, hidden] (projected vision tokens) -> k_norm(K), V into the paged cache at ``slots``."""
        Nv = states.shape[0]
        hk, hd = self.hk, self.hd
        kv = self.kv_proj(states)
        k = self.k_norm(kv[:, :hk * hd].contiguous().view(Nv * hk, hd)).view(Nv, hk, hd)
        v = kv[:, hk * hd:].contiguous().view(Nv, hk, hd)
        ops.kv_write(k, v, k_cache, v_cache, slots)

    def forward(self, x, batch: Batch, k_cache, v_cache, residual, rms_eps):
        T = x.shape[0]
        h, hd = self.h, self.hd
        q = self.q_proj(x, rms_eps=rms_eps)
        q = self.q_norm(q.view(T * h, hd)).view(T, h, hd)
        zero = torch.zeros((), dtype=q.dtype, device=q.device)
        if batch.is_prefill:
            qb = q.view(batch.B, batch.S, h, hd)
            o = ops.paged_attention(qb, k_cache, v_cache, batch.cross_bt, batch.cross_lens, batch.q_lens,
                                    self.scale, causal=False)
            if batch.cross_pre_lens is not None:  # rows before <|image|>: attend to every tile
                o2 = ops.paged_attention(qb, k_cache, v_cache, batch.cross_bt, batch.cross_full_lens,
                                         batch.cross_pre_lens, self.scale, causal=False)
                o = torch.where(batch.cross_pre_rows.view(batch.B, batch.S, 1, 1), o2, o)
            o = o.reshape(T, h * hd)
        else:
            o = ops.decode_attention(q, k_cache, v_cache, batch.cross_bt, batch.cross_lens, self.scale,
                                     num_splits=batch.cross_splits).view(T, h * hd)
        o = torch.where(batch.cross_attn_rows.view(T, 1), o, zero)
        return self.o_proj(o, residual=residual)   # tanh(attn gate) folded into o_proj


class CrossDecoderLayer(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.cross_attn = CrossAttention(cfg)
        self.input_layernorm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps)
        self.cross_attn_attn_gate = nn.Parameter(torch.zeros(1), requires_grad=False)
        self.mlp = LlamaMLP(cfg)
        self.post_attention_layernorm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps)
        self.cross_attn_mlp_gate = nn.Parameter(torch.zeros(1), requires_grad=False)
        self._gates_folded = False

    @torch.no_grad()
    def fold(self):
        def fold_norm(w, norm):
            w.copy_((w.float() * norm.weight.float()[None, :]).to(w.dtype))
            norm.weight.fill_(1.0)
        fold_norm(self.cross_attn.q_proj.weight, self.input_layernorm)
        fold_norm(self.mlp.gate_up_proj.weight, self.post_attention_layernorm)
        if not self._gates_folded:
            for w, g in ((self.cross_attn.o_proj.weight, self.cross_attn_attn_gate),
                         (self.mlp.down_proj.weight, self.cross_attn_mlp_gate)):
                w.copy_((w.float() * torch.tanh(g.float())).to(w.dtype))
                g.fill_(float("inf"))   # tanh(inf) == 1: re-folding a folded state dict is a no-op
            self._gates_folded = True

    def forward(self, x, batch, kc, vc, cos, sin, folded: bool = True):
        x = self.cross_attn(x, batch, kc, vc, residual=x, rms_eps=self.input_layernorm.eps)
        hmid = self.mlp.gate_up_proj(x, rms_eps=self.post_attention_layernorm.eps)
        hmid = torch.where(batch.cross_mlp_rows.view(-1, 1), hmid,
                           torch.zeros((), dtype=hmid.dtype, device=hmid.device))
        return self.mlp.down_proj(hmid, residual=x)     # tanh(mlp gate) folded into down_proj


class MllamaForConditionalGeneration(LlamaForCausalLM):
    """Text decoder (self + cross layers) with the vision tower and projector attached."""

    def __init__(self, mcfg: MllamaConfig):
        nn.Module.__init__(self)
        cfg = mcfg.text
        self.mcfg = mcfg
        self.cfg = cfg
        self.embed_tokens = VocabParallelEmbedding(cfg.vocab_size + 8, cfg.hidden_size)
        self.cross_layers = tuple(mcfg.cross_attention_layers)
        self.layers = nn.ModuleList([CrossDecoderLayer(cfg) if i in self.cross_layers else LlamaDecoderLayer(cfg)
                                     for i in range(cfg.num_hidden_layers)])
        self.norm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps)
        self.lm_head = ParallelLMHead(cfg.vocab_size, cfg.hidden_size)
        self.vision_model = MllamaVisionModel(mcfg.vision)
        self.multi_modal_projector = Linear(mcfg.vision.vision_output_dim, cfg.hidden_size, bias=True)
        self._rope = None
        self._folded = False

    @property
    def kv_heads_local(self) -> int:
        for layer in self.layers:
            if isinstance(layer, LlamaDecoderLayer):
                return layer.self_attn.hk
        return self.layers[0].cross_attn.hk

    @property
    def tokens_per_image(self) -> int:
        return self.mcfg.vision.max_num_tiles * self.mcfg.vision.num_patches

    @torch.no_grad()
    def fold_norms(self):
        def fold(w, norm):
            w.copy_((w.float() * norm.weight.float()[None, :]).to(w.dtype))
            norm.weight.fill_(1.0)
        for layer in self.layers:
            if isinstance(layer, CrossDecoderLayer):
                layer.fold()
            else:
                fold(layer.self_attn.qkv_proj.weight, layer.input_layernorm)
                fold(layer.mlp.gate_up_proj.weight, layer.post_attention_layernorm)
        fold(self.lm_head.weight, self.norm)
        for layer in self.vision_model.global_layers:
            layer.fold_gates()
        self._folded = True

    def load_state_dict(self, *args, **kwargs):
        r = nn.Module.load_state_dict(self, *args, **kwargs)
        for m in self.modules():
            if hasattr(m, "_gates_folded"):
                m._gates_folded = False
        self._folded = False
        return r

    @torch.no_grad()
    def encode_images(self, pixel_values, aspect_ratio_ids, num_tiles) -> torch.Tensor:
        """pixel_values [N, T, S, S, 3] -> projected cross-attention states [N, T * P, hidden]."""
        if not self._folded:
            self.fold_norms()
        return self.multi_modal_projector(self.vision_model(pixel_values, aspect_ratio_ids, num_tiles))

    @torch.no_grad()
    def write_cross_kv(self, states: torch.Tensor, kv_caches, slots: torch.Tensor):
        """states [Nv, hidden] (several images concatenated), slots [Nv] -> every cross layer's cache."""
        for i in self.cross_layers:
            kc, vc = kv_caches[i]
            self.layers[i].cross_attn.write_image_kv(states, kc, vc, slots)

    def forward(self, batch: Batch, kv_caches) -> torch.Tensor:
        if not self._folded:
            self.fold_norms()
        cos, sin = self.rope(batch.input_ids.device)
        x = self.embed_tokens(batch.input_ids)
        use_cross = batch.cross_bt is not None
        for i, (layer, (kc, vc)) in enumerate(zip(self.layers, kv_caches)):
            if i in self.cross_layers and not use_cross:
                continue
            x = layer(x, batch, kc, vc, cos, sin, folded=True)
        if batch.is_prefill:
            x = x.index_select(0, batch.last_index)
        return self.lm_head.logits(x, rms_eps=self.norm.eps)

    def convert_hf_state_dict(self, sd: dict) -> dict:
        """transformers Mllama keys (v4 ``language_model.model.*`` or v5 ``model.language_model.*``) -> ours."""
        vis_map = {
            "gated_positional_embedding.embedding": "pos_embedding",
            "gated_positional_embedding.gate": "pos_gate",
            "gated_positional_embedding.tile_embedding.weight": "tile_pos_embedding",
            "pre_tile_positional_embedding.embedding.weight": "pre_tile_embedding",
            "pre_tile_positional_embedding.gate": "pre_tile_gate",
            "post_tile_positional_embedding.embedding.weight": "post_tile_embedding",
            "post_tile_positional_embedding.gate": "post_tile_gate",
        }
        out = {}
        for k, v in sd.items():
            k2 = k[len("model."):] if k.startswith("model.") else k
            if k2.startswith("language_model."):
                k2 = k2[len("language_model."):]
                k2 = k2[len("model."):] if k2.startswith("model.") else k2
            if "rotary_emb" in k2:
                continue
            if k2.startswith("vision_model."):
                rest = k2[len("vision_model."):]
                rest = vis_map.get(rest, rest)
                rest = rest.replace("global_transformer.layers.", "global_layers.")
                rest = rest.replace("transformer.layers.", "layers.")
                rest = rest.replace(".mlp.fc1.", ".fc1.").replace(".mlp.fc2.", ".fc2.")
                k2 = "vision_model." + rest
            out[k2] = v
        if "lm_head.weight" not in out and "embed_tokens.weight" in out:
            out["lm_head.weight"] = out["embed_tokens.weight"][: self.cfg.vocab_size]
        vc = self.mcfg.vision
        for i in range(vc.num_hidden_layers):
            merge_linear_keys(out, f"vision_model.layers.{i}.self_attn.", ["q_proj", "k_proj", "v_proj"], "qkv",
                              bias=False)
        for i in range(vc.num_global_layers):
            merge_linear_keys(out, f"vision_model.global_layers.{i}.self_attn.", ["q_proj", "k_proj", "v_proj"],
                              "qkv", bias=False)
        for i in range(self.cfg.num_hidden_layers):
            p = f"layers.{i}."
            if i in self.cross_layers:
                merge_linear_keys(out, p + "cross_attn.", ["k_proj", "v_proj"], "kv_proj", bias=False)
            else:
                merge_linear_keys(out, p + "self_attn.", ["q_proj", "k_proj", "v_proj"], "qkv_proj", bias=False)
            gk, uk = p + "mlp.gate_proj.weight", p + "mlp.up_proj.weight"
            if gk in out and uk in out:
                out[p + "mlp.gate_up_proj.weight"] = GLULinear.interleave(out.pop(uk), out.pop(gk))
        return out
