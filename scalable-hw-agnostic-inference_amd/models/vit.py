"""ViT image classifier and YOLOS object detector (transformers architectures).

* ``ViTForImageClassification`` -- google/vit-base-patch16-224 served by
  app/run-vit.py:35-71 (vit/vit-g6-deploy.yaml:40-41).
* ``YolosForObjectDetection`` -- hustvl/yolos-tiny served by app/run-yolo.py
  (whose /detectobj handler is broken in the reference, run-yolo.py:68; here it
  works): DeiT-style encoder + 100 detection tokens, interpolated position
  embeddings, class / box MLP heads.

The 16x16 stride-16 patch embedding is the implicit-GEMM conv kernel (input
channels padded 3 -> 8); the pre-LN encoder uses the fused QKV GEMM + flash
attention; images are preprocessed on the GPU (resize + normalise) so the
host does no per-pixel work.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from .attention import FusedSelfAttention, merge_linear_keys
from .layers import Conv2d, LayerNorm, Linear


# LayerNorms folded into the GEMMs that consume them, moments handed over by the producing GEMM (unet2d.py);
# SHAI_NORM_HANDOFF=0 restores the standalone LayerNorm passes
NORM_HANDOFF = os.environ.get("SHAI_NORM_HANDOFF", "1") != "0"


@dataclass
class ViTConfig:
    image_size: Tuple[int, int] = (224, 224)
    patch_size: int = 16
    hidden_size: int = 768
    num_hidden_layers: int = 12
    num_attention_heads: int = 12
    intermediate_size: int = 3072
    layer_norm_eps: float = 1e-12
    num_labels: int = 1000
    hidden_act: str = "gelu"
    image_mean: Tuple[float, ...] = (0.5, 0.5, 0.5)
    image_std: Tuple[float, ...] = (0.5, 0.5, 0.5)
    num_detection_tokens: int = 0        # YOLOS
    id2label: Optional[Dict[int, str]] = None

    @staticmethod
    def vit_base():
        return ViTConfig()

    @staticmethod
    def yolos_tiny():
        return ViTConfig(image_size=(800, 1333), hidden_size=192, num_hidden_layers=12, num_attention_heads=3,
                         intermediate_size=768, num_labels=91, num_detection_tokens=100,
                         image_mean=(0.485, 0.456, 0.406), image_std=(0.229, 0.224, 0.225))

    @staticmethod
    def tiny(detection=False):
        return ViTConfig(image_size=(64, 64), hidden_size=64, num_hidden_layers=2, num_attention_heads=1,
                         intermediate_size=128, num_labels=10, num_detection_tokens=5 if detection else 0)


class ViTLayer(nn.Module):
    def __init__(self, c: ViTConfig):
        super().__init__()
        self.layernorm_before = LayerNorm(c.hidden_size, c.layer_norm_eps)
        self.attention = FusedSelfAttention(c.hidden_size, c.num_attention_heads)
        self.layernorm_after = LayerNorm(c.hidden_size, c.layer_norm_eps)
        self.intermediate = Linear(c.hidden_size, c.intermediate_size)
        self.output = Linear(c.intermediate_size, c.hidden_size)
        self.act = c.hidden_act

    def forward(self, x):
        x = self.attention(self.layernorm_before(x), residual=x)
        return self.output(self.intermediate(self.layernorm_after(x), act=self.act), residual=x)

    def forward_folded(self, x, mr, next_eps=None):
        """forward with both LayerNorms folded into the QKV / fc1 GEMMs (``ops.fold_layernorm``): ``mr`` = (mean,
        rstd) of x's rows, the residual GEMMs hand the next norm's over (``next_eps``: the next layer's eps, None
        for the last layer).  Returns (out, mr or None)."""
        B, T, C = x.shape
        a = self.attention
        w, b, s = a.qkv.folded(self.layernorm_before)
        q, k, v = a.split(ops.linear(x, w, b, row_affine=(mr, s)))
        o = ops.attention(q, k, v).view(B, T, a.heads * a.head_dim)
        x, mr = a.out.forward_stats(o, residual=x, stats="ln", eps=self.layernorm_after.eps)
        w, b, s = self.intermediate.folded(self.layernorm_after)
        h = ops.linear(x, w, b, act=self.act, row_affine=(mr, s))
        if next_eps is None:
            return self.output(h, residual=x), None
        return self.output.forward_stats(h, residual=x, stats="ln", eps=next_eps)

    def forward_cls(self, x, mr=None, keep: int = 1, tail: bool = False):
        """The last layer when only some tokens leave the encoder: the first ``keep`` (token 0, CLS: image
        classification) or, with ``tail``, the last ``keep`` (YOLOS's detection tokens).  K / V of every token, the
        rest -- attention queries, out-projection, MLP -- for the kept tokens only (M = B keep instead of B T).
        ``mr``: x's LayerNorm moments for the folded QKV (None: the plain norm).  Returns [B, keep, d]."""
        B, T, C = x.shape
        sel = slice(T - keep, T) if tail else slice(0, keep)
        a = self.attention
        if mr is not None:
            w, b, s = a.qkv.folded(self.layernorm_before)
            qkv = ops.linear(x, w, b, row_affine=(mr, s))
        else:
            qkv = a.qkv(self.layernorm_before(x))
        q, k, v = a.split(qkv)
        o = ops.attention(q[:, sel], k, v).reshape(B, keep, a.heads * a.head_dim)
        x0 = a.out(o, residual=x[:, sel].contiguous())
        return self.output(self.intermediate(self.layernorm_after(x0), act=self.act), residual=x0)


class ViTEncoderModel(nn.Module):
    def __init__(self, c: ViTConfig):
        super().__init__()
        self.cfg = c
        gh, gw = c.image_size[0] // c.patch_size, c.image_size[1] // c.patch_size
        self.grid = (gh, gw)
        self.patch = Conv2d(3, c.hidden_size, c.patch_size, stride=c.patch_size)
        self.cls_token = nn.Parameter(torch.empty(1, 1, c.hidden_size, dtype=torch.bfloat16), requires_grad=False)
        self.det_tokens = (nn.Parameter(torch.empty(1, c.num_detection_tokens, c.hidden_size, dtype=torch.bfloat16),
                                        requires_grad=False) if c.num_detection_tokens else None)
        n_pos = 1 + gh * gw + c.num_detection_tokens
        self.position_embeddings = nn.Parameter(torch.empty(1, n_pos, c.hidden_size, dtype=torch.bfloat16),
                                                requires_grad=False)
        self.layers = nn.ModuleList([ViTLayer(c) for _ in range(c.num_hidden_layers)])
        self.layernorm = LayerNorm(c.hidden_size, c.layer_norm_eps)

    def _kept(self, cls_only: bool):
        return (1, False) if cls_only else (self.cfg.num_detection_tokens, True)

    def pos_embed(self, gh: int, gw: int) -> torch.Tensor:
        """Position embeddings for a (gh, gw) patch grid (bicubic interpolation of the
        trained grid, YOLOS InterpolateInitialPositionEmbeddings semantics)."""
        pe = self.position_embeddings
        if (gh, gw) == self.grid:
            return pe
        nd = self.cfg.num_detection_tokens
        cls_pe = pe[:, :1]
        det_pe = pe[:, pe.shape[1] - nd:] if nd else pe[:, :0]
        patch = pe[:, 1:pe.shape[1] - nd].float()
        H0, W0 = self.grid
        patch = patch.transpose(1, 2).reshape(1, -1, H0, W0)
        patch = F.interpolate(patch, size=(gh, gw), mode="bicubic", align_corners=False)
        patch = patch.flatten(2).transpose(1, 2).to(pe.dtype)
        return torch.cat([cls_pe, patch, det_pe], dim=1)

    def forward(self, pixels: torch.Tensor, cls_only: bool = False, det_only: bool = False) -> torch.Tensor:
        """pixels NHWC [B, H, W, 3] normalised bf16 -> hidden states [B, T, d]; ``cls_only``: [B, 1, d] of token 0,
        ``det_only``: [B, nd, d] of the detection tokens -- the last layer then runs its query side for those tokens
        only (``ViTLayer.forward_cls``)."""
        B, H, W, _ = pixels.shape
        x = self.patch(pixels)  # [B, gh, gw, d]
        gh, gw = x.shape[1], x.shape[2]
        toks = [self.cls_token.expand(B, -1, -1), x.reshape(B, gh * gw, -1)]
        if self.det_tokens is not None:
            toks.append(self.det_tokens.expand(B, -1, -1))
        x = torch.cat(toks, dim=1)
        pe = self.pos_embed(gh, gw).expand(B, -1, -1).contiguous()
        x = ops.bias_act(x.contiguous(), None, pe)
        c = self.cfg
        if NORM_HANDOFF and ops.fold_profitable(x.shape[0] * x.shape[1], min(3 * c.hidden_size, c.intermediate_size)):
            layers = list(self.layers)
            mr = ops.row_moments(x, layers[0].layernorm_before.eps)
            for i, layer in enumerate(layers):
                if (cls_only or det_only) and i + 1 == len(layers):
                    return self.layernorm(layer.forward_cls(x, mr, *self._kept(cls_only)))
                nxt = layers[i + 1].layernorm_before.eps if i + 1 < len(layers) else None
                x, mr = layer.forward_folded(x, mr, nxt)
            return self.layernorm(x)
        for i, layer in enumerate(self.layers):
            if (cls_only or det_only) and i + 1 == len(self.layers):
                return self.layernorm(layer.forward_cls(x, None, *self._kept(cls_only)))
            x = layer(x)
        return self.layernorm(x)


def preprocess(images_u8: torch.Tensor, size: Tuple[int, int], mean, std, device) -> torch.Tensor:
    """uint8 NHWC (or list of HWC) -> resized, normalised NHWC bf16 on device."""
    x = images_u8.to(device).permute(0, 3, 1, 2).float() / 255.0
    x = F.interpolate(x, size=size, mode="bilinear", align_corners=False, antialias=x.shape[-1] > size[1])
    m = torch.tensor(mean, device=device).view(1, 3, 1, 1)
    s = torch.tensor(std, device=device).view(1, 3, 1, 1)
    return ((x - m) / s).permute(0, 2, 3, 1).contiguous().to(torch.bfloat16)


def _convert_vit_keys(sd: dict, prefix: str, n_layers: int) -> dict:
    out = {}
    for k, v in sd.items():
        k2 = k[len(prefix):] if k.startswith(prefix) else k
        k2 = k2.replace("embeddings.patch_embeddings.projection", "patch")
        k2 = k2.replace("embeddings.cls_token", "cls_token").replace("embeddings.detection_tokens", "det_tokens")
        k2 = k2.replace("embeddings.position_embeddings", "position_embeddings")
        k2 = k2.replace("encoder.layer.", "layers.")
        k2 = k2.replace("attention.output.dense", "attention.out")
        k2 = k2.replace("attention.attention.query", "attention.query").replace("attention.attention.key",
                                                                                "attention.key")
        k2 = k2.replace("attention.attention.value", "attention.value")
        k2 = k2.replace("intermediate.dense", "intermediate").replace("output.dense", "output")
        # transformers >= 5 naming (vit.layers.N.attention.{q,k,v,o}_proj, mlp.fc1/fc2)
        k2 = k2.replace("attention.q_proj", "attention.query").replace("attention.k_proj", "attention.key")
        k2 = k2.replace("attention.v_proj", "attention.value").replace("attention.o_proj", "attention.out")
        k2 = k2.replace("mlp.fc1", "intermediate").replace("mlp.fc2", "output")
        if "mid_position_embeddings" in k2:
            continue
        out[k2] = v
    for i in range(n_layers):
        merge_linear_keys(out, f"layers.{i}.attention.", ["query", "key", "value"], "qkv")
    return out


class ViTForImageClassification(nn.Module):
    def __init__(self, cfg: ViTConfig = None):
        super().__init__()
        self.cfg = cfg or ViTConfig()
        self.vit = ViTEncoderModel(self.cfg)
        self.classifier = Linear(self.cfg.hidden_size, self.cfg.num_labels)

    def forward(self, pixels):
        h = self.vit(pixels, cls_only=True)  # the logits read token 0 only
        return self.classifier(h[:, 0].contiguous())

    def convert_hf_state_dict(self, sd: dict) -> dict:
        out = {}
        for k, v in sd.items():
            if k.startswith("classifier."):
                out[k] = v
            else:
                out.update({"vit." + kk: vv for kk, vv in _convert_vit_keys({k: v}, "vit.", 0).items()})
        for i in range(self.cfg.num_hidden_layers):
            merge_linear_keys(out, f"vit.layers.{i}.attention.", ["query", "key", "value"], "qkv")
        return out


class MLPHead(nn.Module):
    def __init__(self, din, hidden, dout, n):
        super().__init__()
        dims = [din] + [hidden] * (n - 1) + [dout]
        self.layers = nn.ModuleList([Linear(dims[i], dims[i + 1]) for i in range(n)])

    def forward(self, x):
        for i, l in enumerate(self.layers):
            x = l(x, act="relu" if i < len(self.layers) - 1 else None)
        return x


class YolosForObjectDetection(nn.Module):
    def __init__(self, cfg: ViTConfig = None):
        super().__init__()
        self.cfg = cfg or ViTConfig.yolos_tiny()
        c = self.cfg
        self.vit = ViTEncoderModel(c)
        self.class_labels_classifier = MLPHead(c.hidden_size, c.hidden_size, c.num_labels + 1, 3)
        self.bbox_predictor = MLPHead(c.hidden_size, c.hidden_size, 4, 3)

    def forward(self, pixels):
        """-> (logits [B, 100, num_labels+1], boxes [B, 100, 4] (cx, cy, w, h) in [0, 1])."""
        det = self.vit(pixels, det_only=True).contiguous()  # the heads read the detection tokens only
        logits = self.class_labels_classifier(det)
        boxes = torch.sigmoid(self.bbox_predictor(det).float())
        return logits, boxes

    @staticmethod
    def postprocess(logits, boxes, sizes: List[Tuple[int, int]], threshold: float = 0.5, id2label=None):
        """HF object-detection pipeline output format per image."""
        probs = torch.softmax(logits.float(), -1)[..., :-1]
        scores, labels = probs.max(-1)
        out = []
        for b, (h, w) in enumerate(sizes):
            dets = []
            for s, l, bx in zip(scores[b].tolist(), labels[b].tolist(), boxes[b].float().tolist()):
                if s < threshold:
                    continue
                cx, cy, bw, bh = bx
                dets.append({"score": round(s, 4), "label": (id2label or {}).get(l, f"LABEL_{l}"),
                             "box": {"xmin": int((cx - bw / 2) * w), "ymin": int((cy - bh / 2) * h),
                                     "xmax": int((cx + bw / 2) * w), "ymax": int((cy + bh / 2) * h)}})
            out.append(sorted(dets, key=lambda d: -d["score"]))
        return out

    def convert_hf_state_dict(self, sd: dict) -> dict:
        out = {}
        for k, v in sd.items():
            if k.startswith("class_labels_classifier.") or k.startswith("bbox_predictor."):
                out[k] = v
            else:
                out.update({"vit." + kk: vv for kk, vv in _convert_vit_keys({k: v}, "vit.", 0).items()})
        for i in range(self.cfg.num_hidden_layers):
            merge_linear_keys(out, f"vit.layers.{i}.attention.", ["query", "key", "value"], "qkv")
        return out
