"""CLIP text encoder (transformers ``CLIPTextModel`` architecture).

Used by SD2.1 (OpenCLIP-H text tower: d=1024, 23 layers, 16 heads, GELU) and by
Flux.1 (CLIP-L: d=768, 12 layers, quick-GELU, pooled EOS output).  Reference:
the text encoder the SD/Flux pipelines run (app/run-sd.py:104-135 via diffusers;
app/src/text_encoder_1/model.py:8-33 traced for Neuron).

Pre-LN transformer, causal self-attention on the fused flash kernel, fused QKV
GEMM, residual adds in the GEMM epilogues.  Weight names follow transformers so
HF safetensors load via :meth:`convert_hf_state_dict`.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.nn as nn

from .. import ops
from .attention import FusedSelfAttention, merge_linear_keys
from .layers import Embedding, LayerNorm, Linear


@dataclass
class CLIPTextConfig:
    vocab_size: int = 49408
    hidden_size: int = 1024
    intermediate_size: int = 4096
    num_hidden_layers: int = 23
    num_attention_heads: int = 16
    max_position_embeddings: int = 77
    hidden_act: str = "gelu"
    layer_norm_eps: float = 1e-5
    bos_token_id: int = 49406
    eos_token_id: int = 49407
    pad_token_id: int = 0

    @staticmethod
    def sd21():
        return CLIPTextConfig()

    @staticmethod
    def clip_l():
        return CLIPTextConfig(hidden_size=768, intermediate_size=3072, num_hidden_layers=12, num_attention_heads=12,
                              hidden_act="quick_gelu", pad_token_id=49407)

    @staticmethod
    def tiny():
        return CLIPTextConfig(vocab_size=1000, hidden_size=128, intermediate_size=256, num_hidden_layers=2,
                              num_attention_heads=2, bos_token_id=998, eos_token_id=999)


class CLIPMLP(nn.Module):
    def __init__(self, cfg: CLIPTextConfig):
        super().__init__()
        self.act = cfg.hidden_act
        self.fc1 = Linear(cfg.hidden_size, cfg.intermediate_size)
        self.fc2 = Linear(cfg.intermediate_size, cfg.hidden_size)

    def forward(self, x, residual):
        return self.fc2(self.fc1(x, act=self.act), residual=residual)


class CLIPEncoderLayer(nn.Module):
    def __init__(self, cfg: CLIPTextConfig):
        super().__init__()
        self.layer_norm1 = LayerNorm(cfg.hidden_size, cfg.layer_norm_eps)
        self.self_attn = FusedSelfAttention(cfg.hidden_size, cfg.num_attention_heads)
        self.layer_norm2 = LayerNorm(cfg.hidden_size, cfg.layer_norm_eps)
        self.mlp = CLIPMLP(cfg)

    def forward(self, x, kv_lens=None):
        x = self.self_attn(self.layer_norm1(x), residual=x, causal=True, kv_lens=kv_lens)
        return self.mlp(self.layer_norm2(x), residual=x)


class CLIPTextModel(nn.Module):
    def __init__(self, cfg: CLIPTextConfig = None):
        super().__init__()
        cfg = cfg or CLIPTextConfig()
        self.cfg = cfg
        self.token_embedding = Embedding(cfg.vocab_size, cfg.hidden_size)
        self.position_embedding = nn.Parameter(torch.empty(cfg.max_position_embeddings, cfg.hidden_size,
                                                           dtype=torch.bfloat16), requires_grad=False)
        self.layers = nn.ModuleList([CLIPEncoderLayer(cfg) for _ in range(cfg.num_hidden_layers)])
        self.final_layer_norm = LayerNorm(cfg.hidden_size, cfg.layer_norm_eps)

    def forward(self, input_ids: torch.Tensor, output_pooled: bool = False):
        """input_ids [B, 77] -> last_hidden_state [B, 77, d] (and pooled EOS state)."""
        B, T = input_ids.shape
        x = self.token_embedding(input_ids)
        x = ops.bias_act(x, None, self.position_embedding[:T].expand(B, T, -1).contiguous()) if x.is_cuda \
            else x + self.position_embedding[:T]
        for layer in self.layers:
            x = layer(x)
        x = self.final_layer_norm(x)
        if not output_pooled:
            return x
        if self.cfg.eos_token_id == 2:
            eos = input_ids.argmax(-1)
        else:
            eos = (input_ids == self.cfg.eos_token_id).int().argmax(-1)
        pooled = x[torch.arange(B, device=x.device), eos]
        return x, pooled

    @staticmethod
    def convert_hf_state_dict(sd: dict) -> dict:
        """transformers CLIPTextModel keys -> this module's keys (fused QKV)."""
        out = {}
        for k, v in sd.items():
            k2 = k
            for pre in ("text_model.", "model."):
                if k2.startswith(pre):
                    k2 = k2[len(pre):]
            k2 = k2.replace("embeddings.token_embedding.", "token_embedding.")
            k2 = k2.replace("embeddings.position_embedding.weight", "position_embedding")
            k2 = k2.replace("encoder.layers.", "layers.")
            k2 = k2.replace("self_attn.out_proj.", "self_attn.out.")
            if "position_ids" in k2 or k2.startswith("text_projection"):
                continue
            out[k2] = v
        n = max([int(k.split(".")[1]) for k in out if k.startswith("layers.")] + [-1]) + 1
        for i in range(n):
            merge_linear_keys(out, f"layers.{i}.self_attn.", ["q_proj", "k_proj", "v_proj"], "qkv")
        return out
