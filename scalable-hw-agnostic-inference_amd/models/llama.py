"""Llama-family decoder (Llama-3 8B/70B, Mistral-7B-v0.3, DeepSeek-R1-Distill-Llama-70B).

Serves the reference's LLM endpoints (app/vllm_model_api.py, app/run-llama.py,
app/deepseek_model_api.py; vLLM / NeuronModelForCausalLM underneath).
MI355X-first:

* Paged KV cache ([blocks, Hkv, 64, hd] per layer) written by ``ops.kv_write``;
  prefill attention = flash kernel over the paged cache (so chunked prefill and
  prefix reuse are the same code path); decode = split-K paged decode kernel.
* Fused QKV GEMM, RoPE kernel on strided q/k views, SwiGLU fused into the
  gate/up GEMM epilogue, residual-add fused into RMSNorm.
* Tensor parallel over RCCL: QKV/gate-up column-sharded by heads /
  intermediate, o_proj/down row-sharded with one all-reduce each, vocab-
  parallel embedding + LM head.  bf16 weights (288 GB HBM makes 4-bit
  quantisation, app/run-llama.py:25, unnecessary for capacity).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field
from typing import List, Optional

import torch
import torch.nn as nn

from .. import ops
from ..parallel.layers import (GLUParallelLinear, ParallelLMHead, QKVParallelLinear, RowParallelLinear,
                               VocabParallelEmbedding)
from ..parallel.state import tp
from .layers import GLULinear, RMSNorm

# decode steps run RoPE + the KV-cache write inside the paged decode-attention kernel (one launch per layer
# instead of two); SHAI_FUSED_DECODE=0 keeps the separate rope_qkv_cache launch
FUSED_DECODE = os.environ.get("SHAI_FUSED_DECODE", "1") != "0"
# decode with the norm folded into qkv_proj: the QKV GEMM's split-K fold runs inside the attention kernel
# (one launch fewer per layer); SHAI_QKV_FOLD_IN_ATTN=0 keeps the GEMM's own fold launch
QKV_FOLD_IN_ATTN = os.environ.get("SHAI_QKV_FOLD_IN_ATTN", "1") != "0"
# ... only up to this many decode-attention splits: every split workgroup of a (row, KV head) re-reads all the
# partial slabs, so at long contexts (decode_splits raises the count to 16-64) the separate fold is cheaper
QKV_FOLD_MAX_SPLITS = int(os.environ.get("SHAI_QKV_FOLD_MAX_SPLITS", "8"))

KV_BLOCK = 64


@dataclass
class LlamaConfig:
    vocab_size: int = 32768
    hidden_size: int = 4096
    intermediate_size: int = 14336
    num_hidden_layers: int = 32
    num_attention_heads: int = 32
    num_key_value_heads: int = 8
    head_dim: int = 128
    rms_norm_eps: float = 1e-5
    rope_theta: float = 1e6
    max_position_embeddings: int = 32768
    tie_word_embeddings: bool = False
    bos_token_id: int = 1
    eos_token_id: int = 2
    rope_scaling: Optional[dict] = None

    @staticmethod
    def mistral_7b():
        return LlamaConfig()

    @staticmethod
    def llama3_8b():
        return LlamaConfig(vocab_size=128256, rope_theta=5e5, max_position_embeddings=8192, bos_token_id=128000,
                           eos_token_id=128001)

    @staticmethod
    def llama31_8b():
        """Llama-3.1-8B: the 128k-context text model (and the Llama-3.2-11B-Vision text tower's shape), llama3
        RoPE scaling."""
        c = LlamaConfig.llama3_8b()
        c.max_position_embeddings = 131072
        c.rope_scaling = {"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0, "high_freq_factor": 4.0,
                          "original_max_position_embeddings": 8192}
        return c

    @staticmethod
    def llama3_70b():
        return LlamaConfig(vocab_size=128256, hidden_size=8192, intermediate_size=28672, num_hidden_layers=80,
                           num_attention_heads=64, num_key_value_heads=8, rope_theta=5e5,
                           max_position_embeddings=8192, bos_token_id=128000, eos_token_id=128001)

    @staticmethod
    def deepseek_r1_distill_70b():
        c = LlamaConfig.llama3_70b()
        c.max_position_embeddings = 131072
        c.rope_scaling = {"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0, "high_freq_factor": 4.0,
                          "original_max_position_embeddings": 8192}
        return c

    @staticmethod
    def tiny():
        return LlamaConfig(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                           num_attention_heads=4, num_key_value_heads=2, head_dim=64, max_position_embeddings=1024)

    @staticmethod
    def from_hf(d: dict) -> "LlamaConfig":
        hd = d.get("head_dim") or d["hidden_size"] // d["num_attention_heads"]
        return LlamaConfig(vocab_size=d["vocab_size"], hidden_size=d["hidden_size"],
                           intermediate_size=d["intermediate_size"], num_hidden_layers=d["num_hidden_layers"],
                           num_attention_heads=d["num_attention_heads"],
                           num_key_value_heads=d.get("num_key_value_heads", d["num_attention_heads"]), head_dim=hd,
                           rms_norm_eps=d.get("rms_norm_eps", 1e-5), rope_theta=d.get("rope_theta", 1e4),
                           max_position_embeddings=d.get("max_position_embeddings", 4096),
                           tie_word_embeddings=d.get("tie_word_embeddings", False),
                           bos_token_id=d.get("bos_token_id", 1) or 1,
                           eos_token_id=(d.get("eos_token_id", 2) if not isinstance(d.get("eos_token_id"), list)
                                         else d["eos_token_id"][0]),
                           rope_scaling=d.get("rope_scaling"))


def rope_tables(cfg: LlamaConfig, max_pos: int, device) -> tuple:
    hd = cfg.head_dim
    inv = 1.0 / (cfg.rope_theta ** (torch.arange(0, hd, 2, dtype=torch.float64) / hd))
    rs = cfg.rope_scaling
    if rs and rs.get("rope_type", rs.get("type")) == "llama3":
        factor, lf, hf = rs["factor"], rs["low_freq_factor"], rs["high_freq_factor"]
        old = rs["original_max_position_embeddings"]
        wavelen = 2 * math.pi / inv
        low_wl, high_wl = old / lf, old / hf
        smooth = (old / wavelen - lf) / (hf - lf)
        scaled = torch.where(wavelen > low_wl, inv / factor, inv)
        mid = (1 - smooth) * inv / factor + smooth * inv
        inv = torch.where((wavelen <= low_wl) & (wavelen >= high_wl), mid, scaled)
    t = torch.arange(max_pos, dtype=torch.float64)
    fr = torch.outer(t, inv)
    return fr.cos().float().to(device).contiguous(), fr.sin().float().to(device).contiguous()


@dataclass
class Batch:
    """Flattened token batch for one engine step (prefill: packed varlen rows, or padded to [B, S])."""
    input_ids: torch.Tensor         # [T] int32 (T = B*S for prefill, B for decode)
    positions: torch.Tensor         # [T] int32
    slots: torch.Tensor             # [T] int32 cache slot (-1 = padding)
    block_table: torch.Tensor       # [B, max_blocks] int32
    ctx_lens: torch.Tensor          # [B] int32 (context length incl. this step's tokens)
    q_lens: Optional[torch.Tensor]  # [B] int32 (prefill only)
    B: int
    S: int                          # tokens per sequence in this step (1 for decode)
    is_prefill: bool
    num_splits: int = 1             # decode split-K
    last_index: Optional[torch.Tensor] = None  # [B] flat index of each sequence's last token (prefill)
    # cross-attention to image K/V (Llama-3.2-Vision; see models/mllama.py), None for text-only steps
    cross_bt: Optional[torch.Tensor] = None         # [B, max_cross_blocks] int32 image K/V blocks
    cross_lens: Optional[torch.Tensor] = None       # [B] int32 valid-tile image tokens (>= 1)
    cross_full_lens: Optional[torch.Tensor] = None  # [B] int32 all-tile image tokens (rows before <|image|>)
    cross_pre_lens: Optional[torch.Tensor] = None   # [B] int32 rows before <|image|> (prefill; None if none)
    cross_pre_rows: Optional[torch.Tensor] = None   # [T] bool row is before <|image|>
    cross_attn_rows: Optional[torch.Tensor] = None  # [T] bool row's sequence has an image
    cross_mlp_rows: Optional[torch.Tensor] = None   # [T] bool cross MLP applies (image, at/after <|image|>)
    cross_splits: int = 1
    # packed varlen prefill: T = sum(q_lens) rows, sequence b's rows start at q_start[b] (no padding rows);
    # S is then max(q_lens).  None = the padded [B, S] layout.
    q_start: Optional[torch.Tensor] = None


class LlamaAttention(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        st = tp()
        self.cfg = cfg
        self.qkv_proj = QKVParallelLinear(cfg.hidden_size, cfg.num_attention_heads, cfg.num_key_value_heads,
                                          cfg.head_dim)
        self.o_proj = RowParallelLinear(cfg.num_attention_heads * cfg.head_dim, cfg.hidden_size, bias=False)
        self.h = self.qkv_proj.h_local
        self.hk = self.qkv_proj.kv_local
        self.hd = cfg.head_dim
        self.scale = 1.0 / math.sqrt(cfg.head_dim)

    def forward(self, x, batch: Batch, k_cache, v_cache, cos, sin, residual=None, rms_eps=None):
        T = x.shape[0]
        h, hk, hd = self.h, self.hk, self.hd
        qp = self.qkv_proj
        if (not batch.is_prefill and FUSED_DECODE and QKV_FOLD_IN_ATTN and rms_eps is not None and x.is_cuda
                and (batch.num_splits or 1) <= QKV_FOLD_MAX_SPLITS and T <= 64 and qp.bias is None and qp.w_scale is None and qp.weight.dtype == torch.bfloat16
                and x.is_contiguous() and x.shape[1] >= 2048):
            o = ops.decode_attention_rope_qkv(x, qp.weight, rms_eps, k_cache, v_cache, batch.block_table,
                                              batch.ctx_lens, batch.positions, cos, sin, batch.slots, h, hk,
                                              self.scale, num_splits=batch.num_splits)
            return self.o_proj(o, residual=residual)
        qkv = qp(x, rms_eps=rms_eps)  # [T, (h + 2hk) * hd]
        if not batch.is_prefill and FUSED_DECODE:  # RoPE + KV-cache write inside the decode attention kernel
            o = ops.decode_attention_rope(qkv, k_cache, v_cache, batch.block_table, batch.ctx_lens, batch.positions,
                                          cos, sin, batch.slots, h, hk, self.scale, num_splits=batch.num_splits)
            return self.o_proj(o, residual=residual)
        ops.rope_qkv_cache(qkv, batch.positions, cos, sin, k_cache, v_cache, batch.slots, h, hk)
        q = qkv[:, : h * hd].view(T, h, hd)
        if batch.is_prefill and batch.q_start is not None:
            o = ops.paged_attention_varlen(q, k_cache, v_cache, batch.block_table, batch.ctx_lens, batch.q_lens,
                                           batch.q_start, batch.S, self.scale).view(T, h * hd)
        elif batch.is_prefill:
            o = ops.paged_attention(q.view(batch.B, batch.S, h, hd), k_cache, v_cache, batch.block_table,
                                    batch.ctx_lens, batch.q_lens, self.scale, causal=True).view(T, h * hd)
        else:
            o = ops.decode_attention(q, k_cache, v_cache, batch.block_table, batch.ctx_lens, self.scale,
                                     num_splits=batch.num_splits).view(T, h * hd)
        return self.o_proj(o, residual=residual)


class LlamaMLP(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.gate_up_proj = GLUParallelLinear(cfg.hidden_size, cfg.intermediate_size, act="silu")
        self.down_proj = RowParallelLinear(cfg.intermediate_size, cfg.hidden_size, bias=False)

    def forward(self, x, residual=None, rms_eps=None):
        return self.down_proj(self.gate_up_proj(x, rms_eps=rms_eps), residual=residual)


class LlamaDecoderLayer(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.input_layernorm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps)
        self.self_attn = LlamaAttention(cfg)
        self.post_attention_layernorm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps)
        self.mlp = LlamaMLP(cfg)

    def forward(self, x, batch, kc, vc, cos, sin, folded: bool = False):
        if folded:  # norm gains live in the qkv / gate_up weights; RMS scaling fused into those GEMMs
            eps = self.input_layernorm.eps
            x = self.self_attn(x, batch, kc, vc, cos, sin, residual=x, rms_eps=eps)
            return self.mlp(x, residual=x, rms_eps=self.post_attention_layernorm.eps)
        x = self.self_attn(self.input_layernorm(x), batch, kc, vc, cos, sin, residual=x)
        return self.mlp(self.post_attention_layernorm(x), residual=x)


class LlamaForCausalLM(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.cfg = cfg
        self.embed_tokens = VocabParallelEmbedding(cfg.vocab_size, cfg.hidden_size)
        self.layers = nn.ModuleList([LlamaDecoderLayer(cfg) for _ in range(cfg.num_hidden_layers)])
        self.norm = RMSNorm(cfg.hidden_size, cfg.rms_norm_eps)
        self.lm_head = ParallelLMHead(cfg.vocab_size, cfg.hidden_size)
        self._rope = None
        self._folded = False

    @torch.no_grad()
    def fold_norms(self):
        """Pre-multiply every RMSNorm gain into the columns of the GEMM that consumes it
        (input_layernorm -> qkv_proj, post_attention_layernorm -> gate_up_proj, norm -> lm_head)
        and reset the gains to 1.  The forward then feeds the raw residual stream to those GEMMs
        with ``rms_eps`` set: on the GPU the per-row 1/rms is computed from the activation tiles
        already streaming through the decode GEMM, so the two norm kernels per layer disappear."""
        def fold(lin_w, norm):
            if lin_w.dtype == torch.float8_e4m3fn:
                raise RuntimeError("fold_norms after fp8 quantisation: fold first, then quantize_fp8_")
            lin_w.copy_((lin_w.float() * norm.weight.float()[None, :]).to(lin_w.dtype))
            norm.weight.fill_(1.0)
        for layer in self.layers:
            fold(layer.self_attn.qkv_proj.weight, layer.input_layernorm)
            fold(layer.mlp.gate_up_proj.weight, layer.post_attention_layernorm)
        fold(self.lm_head.weight, self.norm)
        self._folded = True

    def load_state_dict(self, *args, **kwargs):
        r = super().load_state_dict(*args, **kwargs)
        self._folded = False   # fresh (unfolded) weights: fold again before the next forward
        return r

    @property
    def kv_heads_local(self) -> int:
        return self.layers[0].self_attn.hk

    def rope(self, device):
        if self._rope is None or self._rope[0].device != torch.device(device):
            self._rope = rope_tables(self.cfg, self.cfg.max_position_embeddings, device)
        return self._rope

    def forward(self, batch: Batch, kv_caches: List[tuple]) -> torch.Tensor:
        """Returns logits [B, V] for each sequence's last token of this step."""
        if not self._folded:
            self.fold_norms()
        cos, sin = self.rope(batch.input_ids.device)
        x = self.embed_tokens(batch.input_ids)
        for layer, (kc, vc) in zip(self.layers, kv_caches):
            x = layer(x, batch, kc, vc, cos, sin, folded=True)
        if batch.is_prefill:
            x = x.index_select(0, batch.last_index)
        return self.lm_head.logits(x, rms_eps=self.norm.eps)

    def convert_hf_state_dict(self, sd: dict) -> dict:
        from .attention import merge_linear_keys
        out = {}
        for k, v in sd.items():
            k2 = k[len("model."):] if k.startswith("model.") else k
            if "rotary_emb" in k2:
                continue
            out[k2] = v
        if "lm_head.weight" not in out and "embed_tokens.weight" in out:
            out["lm_head.weight"] = out["embed_tokens.weight"]
        for i in range(self.cfg.num_hidden_layers):
            p = f"layers.{i}."
            merge_linear_keys(out, p + "self_attn.", ["q_proj", "k_proj", "v_proj"], "qkv_proj", bias=False)
            gk, uk = p + "mlp.gate_proj.weight", p + "mlp.up_proj.weight"
            if gk in out and uk in out:
                out[p + "mlp.gate_up_proj.weight"] = GLULinear.interleave(out.pop(uk), out.pop(gk))
        return out


def allocate_kv_cache(cfg: LlamaConfig, kv_heads_local: int, num_blocks: int, device, dtype=torch.bfloat16):
    """One contiguous allocation [L, 2, blocks, Hkv, 64, hd]; returns list of (k, v) views per layer."""
    buf = torch.empty(cfg.num_hidden_layers, 2, num_blocks, kv_heads_local, KV_BLOCK, cfg.head_dim, dtype=dtype,
                      device=device)
    return buf, [(buf[i, 0], buf[i, 1]) for i in range(cfg.num_hidden_layers)]


def kv_bytes_per_block(cfg: LlamaConfig, kv_heads_local: int) -> int:
    return cfg.num_hidden_layers * 2 * kv_heads_local * KV_BLOCK * cfg.head_dim * 2
