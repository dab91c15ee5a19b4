"""T5 v1.1 encoder (transformers ``T5EncoderModel``): T5-v1.1-large for the
embedding API (app/t5_model_api.py:35-46, mean-pooled last hidden state) and
T5-XXL as Flux.1's text_encoder_2 (app/src/text_encoder_2/model.py).

RMS LayerNorm, unscaled attention with a bucketed relative-position bias
(computed once per sequence length, added inside the flash kernel), gated-GELU
FFN fused into one GEMM epilogue.  Tensor parallel (Flux TP8): Q/K/V
column-sharded by heads, O row-sharded (one all-reduce); wi_0/wi_1 column,
wo row.  Unlike app/src/text_encoder_2/model.py:37-73 (gather_output=True,
attention replicated on every rank), attention here runs head-sharded, so
there is no all-gather at all.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch
import torch.nn as nn

from .. import ops
from ..parallel.layers import GLUParallelLinear, QKVParallelLinear, RowParallelLinear
from ..parallel.state import tp
from .layers import Embedding, GLULinear, RMSNorm


@dataclass
class T5Config:
    vocab_size: int = 32128
    d_model: int = 1024
    d_kv: int = 64
    d_ff: int = 2816
    num_layers: int = 24
    num_heads: int = 16
    relative_attention_num_buckets: int = 32
    relative_attention_max_distance: int = 128
    layer_norm_epsilon: float = 1e-6
    feed_forward_proj: str = "gated-gelu"
    pad_token_id: int = 0
    eos_token_id: int = 1

    @staticmethod
    def v1_1_large():
        return T5Config()

    @staticmethod
    def xxl():
        return T5Config(d_model=4096, d_ff=10240, num_heads=64)

    @staticmethod
    def tiny():
        return T5Config(vocab_size=500, d_model=128, d_ff=256, num_layers=2, num_heads=2)


def relative_position_bucket(rel: torch.Tensor, num_buckets: int, max_distance: int) -> torch.Tensor:
    """Bidirectional T5 bucketing (transformers T5Attention._relative_position_bucket)."""
    num_buckets //= 2
    ret = (rel > 0).long() * num_buckets
    n = rel.abs()
    max_exact = num_buckets // 2
    is_small = n < max_exact
    val_large = max_exact + (torch.log(n.float().clamp(min=1) / max_exact) / math.log(max_distance / max_exact) *
                             (num_buckets - max_exact)).long()
    val_large = torch.minimum(val_large, torch.full_like(val_large, num_buckets - 1))
    return ret + torch.where(is_small, n, val_large)


class T5Block(nn.Module):
    def __init__(self, c: T5Config):
        super().__init__()
        self.c = c
        self.ln_attn = RMSNorm(c.d_model, c.layer_norm_epsilon)
        self.qkv = QKVParallelLinear(c.d_model, c.num_heads, c.num_heads, c.d_kv)
        self.o = RowParallelLinear(c.num_heads * c.d_kv, c.d_model, bias=False)
        self.ln_ff = RMSNorm(c.d_model, c.layer_norm_epsilon)
        act = "gelu_tanh" if "gelu" in c.feed_forward_proj else "relu"
        self.wi = GLUParallelLinear(c.d_model, c.d_ff, act=act)
        self.wo = RowParallelLinear(c.d_ff, c.d_model, bias=False)
        self.h = self.qkv.h_local

    def forward(self, x, bias, lens):
        B, S, _ = x.shape
        h, d = self.h, self.c.d_kv
        qkv = self.qkv(self.ln_attn(x))
        q = qkv[..., : h * d].view(B, S, h, d)
        k = qkv[..., h * d:2 * h * d].view(B, S, h, d)
        v = qkv[..., 2 * h * d:].view(B, S, h, d)
        a = ops.attention(q, k, v, scale=1.0, kv_lens=lens, bias=bias)
        x = self.o(a.view(B, S, h * d), residual=x)
        return self.wo(self.wi(self.ln_ff(x)), residual=x)


class T5EncoderModel(nn.Module):
    def __init__(self, cfg: T5Config = None):
        super().__init__()
        c = cfg or T5Config()
        self.cfg = c
        self.shared = Embedding(c.vocab_size, c.d_model)
        st = tp()
        self.h_local = c.num_heads // st.size
        self.h_start = st.rank * self.h_local
        self.relative_attention_bias = nn.Parameter(
            torch.empty(c.relative_attention_num_buckets, c.num_heads, dtype=torch.bfloat16), requires_grad=False)
        self.blocks = nn.ModuleList([T5Block(c) for _ in range(c.num_layers)])
        self.final_layer_norm = RMSNorm(c.d_model, c.layer_norm_epsilon)
        self._bias_cache = {}

    def position_bias(self, S: int, device) -> torch.Tensor:
        key = (S, str(device))
        b = self._bias_cache.get(key)
        if b is None:
            ctx = torch.arange(S, device=device)
            rel = ctx[None, :] - ctx[:, None]
            buckets = relative_position_bucket(rel, self.cfg.relative_attention_num_buckets,
                                               self.cfg.relative_attention_max_distance)
            tab = self.relative_attention_bias[:, self.h_start:self.h_start + self.h_local]
            b = tab[buckets].permute(2, 0, 1).contiguous()  # [H_local, S, S]
            self._bias_cache[key] = b
        return b

    def forward(self, input_ids: torch.Tensor, attention_mask: torch.Tensor = None) -> torch.Tensor:
        B, S = input_ids.shape
        lens = (attention_mask.sum(-1).to(torch.int32) if attention_mask is not None
                else torch.full((B,), S, dtype=torch.int32, device=input_ids.device))
        x = self.shared(input_ids)
        bias = self.position_bias(S, input_ids.device)
        for blk in self.blocks:
            x = blk(x, bias, lens)
        return self.final_layer_norm(x)

    def convert_hf_state_dict(self, sd: dict) -> dict:
        out = {}
        for k, v in sd.items():
            k2 = k[len("encoder."):] if k.startswith("encoder.") else k
            if k2.startswith("embed_tokens"):
                continue
            out[k2] = v
        if "shared.weight" not in out and "encoder.embed_tokens.weight" in sd:
            out["shared.weight"] = sd["encoder.embed_tokens.weight"]
        rab = "block.0.layer.0.SelfAttention.relative_attention_bias.weight"
        if rab in out:
            out["relative_attention_bias"] = out.pop(rab)
        res = {}
        for k, v in out.items():
            if not k.startswith("block."):
                res[k] = v
        for i in range(self.cfg.num_layers):
            p = f"block.{i}.layer."
            q, kk, vv = (out.get(p + f"0.SelfAttention.{n}.weight") for n in "qkv")
            if q is not None:
                res[f"blocks.{i}.qkv.weight"] = torch.cat([q, kk, vv], 0)
                res[f"blocks.{i}.o.weight"] = out[p + "0.SelfAttention.o.weight"]
                res[f"blocks.{i}.ln_attn.weight"] = out[p + "0.layer_norm.weight"]
                res[f"blocks.{i}.ln_ff.weight"] = out[p + "1.layer_norm.weight"]
                res[f"blocks.{i}.wo.weight"] = out[p + "1.DenseReluDense.wo.weight"]
                if p + "1.DenseReluDense.wi_0.weight" in out:
                    res[f"blocks.{i}.wi.weight"] = GLULinear.interleave(out[p + "1.DenseReluDense.wi_1.weight"],
                                                                        out[p + "1.DenseReluDense.wi_0.weight"])
        return res

    def encode_mean(self, input_ids, attention_mask=None) -> torch.Tensor:
        """t5_model_api.py:35-46 semantics: mean over ALL (padded) positions, fp32."""
        return self.forward(input_ids, attention_mask).float().mean(dim=1)
