"""DistilBERT sequence classifier (transformers ``DistilBertForSequenceClassification``),
the SST-2 sentiment model served by app/run-bert.py:21-52
(distilbert-base-uncased-finetuned-sst-2-english, bert/bert-inf-deploy.yaml:50-53).

Post-LN encoder: fused QKV GEMM -> flash attention with a padding mask (per-row
valid lengths, no [B, S, S] mask tensor) -> out-proj -> residual+LayerNorm
fused; FFN GELU fused in the first GEMM's epilogue.  Runs on the GPU kernels
or, for BASELINE.json's CPU "plumbing" config, on the fp32 CPU path.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict

import torch
import torch.nn as nn

from .. import ops
from .attention import FusedSelfAttention, merge_linear_keys
from .layers import Embedding, LayerNorm, Linear


@dataclass
class DistilBertConfig:
    vocab_size: int = 30522
    dim: int = 768
    n_layers: int = 6
    n_heads: int = 12
    hidden_dim: int = 3072
    max_position_embeddings: int = 512
    num_labels: int = 2
    eps: float = 1e-12
    id2label: Dict[int, str] = field(default_factory=lambda: {0: "NEGATIVE", 1: "POSITIVE"})
    pad_token_id: int = 0
    cls_token_id: int = 101
    sep_token_id: int = 102

    @staticmethod
    def tiny():
        return DistilBertConfig(vocab_size=1000, dim=64, n_layers=2, n_heads=1, hidden_dim=128)


class DistilBertLayer(nn.Module):
    def __init__(self, c: DistilBertConfig):
        super().__init__()
        self.attention = FusedSelfAttention(c.dim, c.n_heads)
        self.sa_layer_norm = LayerNorm(c.dim, c.eps)
        self.lin1 = Linear(c.dim, c.hidden_dim)
        self.lin2 = Linear(c.hidden_dim, c.dim)
        self.output_layer_norm = LayerNorm(c.dim, c.eps)

    def forward(self, x, lens):
        a = self.attention(x, kv_lens=lens)
        x, _ = self.sa_layer_norm(a, residual=x)
        f = self.lin2(self.lin1(x, act="gelu"))
        x, _ = self.output_layer_norm(f, residual=x)
        return x


class DistilBertForSequenceClassification(nn.Module):
    def __init__(self, cfg: DistilBertConfig = None):
        super().__init__()
        c = cfg or DistilBertConfig()
        self.cfg = c
        self.word_embeddings = Embedding(c.vocab_size, c.dim)
        self.position_embeddings = Embedding(c.max_position_embeddings, c.dim)
        self.emb_layer_norm = LayerNorm(c.dim, c.eps)
        self.layers = nn.ModuleList([DistilBertLayer(c) for _ in range(c.n_layers)])
        self.pre_classifier = Linear(c.dim, c.dim)
        self.classifier = Linear(c.dim, c.num_labels)

    def forward(self, input_ids: torch.Tensor, attention_mask: torch.Tensor = None) -> torch.Tensor:
        """input_ids [B, S] (right-padded) -> logits [B, num_labels]."""
        B, S = input_ids.shape
        lens = (attention_mask.sum(-1).to(torch.int32) if attention_mask is not None
                else torch.full((B,), S, dtype=torch.int32, device=input_ids.device))
        pos = torch.arange(S, device=input_ids.device).unsqueeze(0).expand(B, S)
        x, _ = self.emb_layer_norm(self.word_embeddings(input_ids), residual=self.position_embeddings(pos))
        for layer in self.layers:
            x = layer(x, lens)
        cls = x[:, 0].contiguous()
        h = self.pre_classifier(cls, act="relu")
        return self.classifier(h)

    def convert_hf_state_dict(self, sd: dict) -> dict:
        out = {}
        for k, v in sd.items():
            k2 = k.replace("distilbert.", "")
            k2 = k2.replace("embeddings.word_embeddings", "word_embeddings")
            k2 = k2.replace("embeddings.position_embeddings", "position_embeddings")
            k2 = k2.replace("embeddings.LayerNorm", "emb_layer_norm")
            k2 = k2.replace("transformer.layer.", "layers.")
            k2 = k2.replace("attention.out_lin", "attention.out")
            k2 = k2.replace("ffn.lin1", "lin1").replace("ffn.lin2", "lin2")
            if "position_ids" in k2:
                continue
            out[k2] = v
        for i in range(self.cfg.n_layers):
            merge_linear_keys(out, f"layers.{i}.attention.", ["q_lin", "k_lin", "v_lin"], "qkv")
        return out
