"""Megatron-style tensor-parallel layers with shard-on-load.

Semantics match NxD's layers the reference uses for Flux / T5 TP8
(app/src/transformer/model.py:162-447, app/src/text_encoder_2/model.py:34-154):

* ``ColumnParallelLinear``: output features sharded, no forward communication
  (``gather_output=True`` all-gathers along the last dim).
* ``RowParallelLinear``: input features sharded, partial products all-reduced;
  the bias (and an optional residual) are added once after the reduction.
* ``QKVParallelLinear``: fused Q/K/V GEMM, sharded by heads (K/V heads
  replicated when kv_heads < tp).
* ``GLUParallelLinear``: fused gate/up (SwiGLU / GEGLU) with (value, gate) rows
  interleaved, sharded by the intermediate dim -- the activation runs in the
  GEMM epilogue on each shard.
* ``VocabParallelEmbedding`` / ``ParallelLMHead``: vocab-sharded.

Every layer's ``_load_from_state_dict`` accepts the FULL (unsharded) tensor and
slices this rank's shard, so one HF checkpoint serves every TP degree.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn

from .. import ops
from . import comm
from .state import tp


def _div(a: int, b: int) -> int:
    assert a % b == 0, f"{a} not divisible by {b}"
    return a // b


class _ShardLoadMixin:
    def _shard(self, name: str, full: torch.Tensor) -> torch.Tensor:
        raise NotImplementedError

    # ---- fp8 weight-only quantisation (vLLM-style ``quantization: fp8``): the weight becomes
    # OCP e4m3 [N, K] + an fp32 per-row ``weight_scale``; decode GEMMs stream half the bytes.
    def quantize_fp8_(self) -> None:
        if getattr(self, "weight_scale", None) is not None:
            return
        w8, scale = ops.quantize_fp8_rows(self.weight.data)
        self.weight = nn.Parameter(w8, requires_grad=False)
        self.register_buffer("weight_scale", scale)

    @property
    def w_scale(self):
        return getattr(self, "weight_scale", None)

    def _load_from_state_dict(self, state_dict, prefix, *args, **kwargs):
        for name, p in list(self._parameters.items()):
            k = prefix + name
            if k in state_dict and p is not None and state_dict[k].shape != p.shape:
                state_dict[k] = self._shard(name, state_dict[k])
        super()._load_from_state_dict(state_dict, prefix, *args, **kwargs)


class ColumnParallelLinear(_ShardLoadMixin, nn.Module):
    def __init__(self, in_features: int, out_features: int, bias: bool = True, gather_output: bool = False,
                 dtype=torch.bfloat16):
        super().__init__()
        st = tp()
        self.tp_rank, self.tp_size = st.rank, st.size
        self.in_features, self.out_features = in_features, out_features
        self.out_local = _div(out_features, st.size)
        self.gather_output = gather_output
        self.weight = nn.Parameter(torch.empty(self.out_local, in_features, dtype=dtype), requires_grad=False)
        self.bias = nn.Parameter(torch.zeros(self.out_local, dtype=dtype), requires_grad=False) if bias else None

    def _shard(self, name, full):
        return full.narrow(0, self.tp_rank * self.out_local, self.out_local).contiguous()

    def full_shape(self, name):
        return (self.out_features, self.in_features) if name == "weight" else (self.out_features,)

    def forward(self, x, act=None, rms_eps=None):
        y = ops.linear(x, self.weight, self.bias, act=act, rms_eps=rms_eps, w_scale=self.w_scale)
        return comm.all_gather_last(y) if self.gather_output else y


class RowParallelLinear(_ShardLoadMixin, nn.Module):
    def __init__(self, in_features: int, out_features: int, bias: bool = True, input_is_parallel: bool = True,
                 dtype=torch.bfloat16):
        super().__init__()
        st = tp()
        self.tp_rank, self.tp_size = st.rank, st.size
        self.in_features, self.out_features = in_features, out_features
        self.in_local = _div(in_features, st.size)
        self.input_is_parallel = input_is_parallel
        self.weight = nn.Parameter(torch.empty(out_features, self.in_local, dtype=dtype), requires_grad=False)
        self.bias = nn.Parameter(torch.zeros(out_features, dtype=dtype), requires_grad=False) if bias else None

    def _shard(self, name, full):
        if name == "bias":
            return full
        return full.narrow(1, self.tp_rank * self.in_local, self.in_local).contiguous()

    def full_shape(self, name):
        return (self.out_features, self.in_features) if name == "weight" else (self.out_features,)

    def forward(self, x, residual=None):
        if not self.input_is_parallel and self.tp_size > 1:
            x = x.narrow(-1, self.tp_rank * self.in_local, self.in_local).contiguous()
        if self.tp_size == 1:
            return ops.linear(x, self.weight, self.bias, residual=residual, w_scale=self.w_scale)
        rows = x.numel() // x.shape[-1]
        # fused (GEMM into the IPC staging slot, one kernel reduces + adds bias / residual) and, at >= 1024 rows,
        # overlapped (row slab i's reduce runs beside slab i + 1's GEMM); CPU (gloo): the same slab schedule
        y = comm.row_parallel_reduce(x, self.weight, self.bias, residual, self.w_scale,
                                     chunks=comm.overlap_chunks(rows, self.out_features))
        if y is not None:
            return y.view(*x.shape[:-1], self.out_features)
        y = ops.linear(x, self.weight, None, w_scale=self.w_scale)
        comm.all_reduce(y)
        if self.bias is not None or residual is not None:
            y = ops.bias_act(y, self.bias, residual)
        return y


class QKVParallelLinear(_ShardLoadMixin, nn.Module):
    """Fused [q; k; v] projection; rows of the full weight ordered q (H*hd), k (Hk*hd), v (Hk*hd)."""

    def __init__(self, hidden: int, heads: int, kv_heads: int, head_dim: int, bias: bool = False,
                 dtype=torch.bfloat16):
        super().__init__()
        st = tp()
        self.tp_rank, self.tp_size = st.rank, st.size
        self.heads, self.kv_heads, self.head_dim = heads, kv_heads, head_dim
        self.h_local = _div(heads, st.size)
        self.kv_local = max(1, kv_heads // st.size)
        self.kv_replicas = max(1, st.size // kv_heads)
        n = (self.h_local + 2 * self.kv_local) * head_dim
        self.weight = nn.Parameter(torch.empty(n, hidden, dtype=dtype), requires_grad=False)
        self.bias = nn.Parameter(torch.zeros(n, dtype=dtype), requires_grad=False) if bias else None

    def _shard(self, name, full):
        hd = self.head_dim
        q = full[: self.heads * hd]
        k = full[self.heads * hd:(self.heads + self.kv_heads) * hd]
        v = full[(self.heads + self.kv_heads) * hd:]
        qs = q.narrow(0, self.tp_rank * self.h_local * hd, self.h_local * hd)
        kv_idx = self.tp_rank // self.kv_replicas
        ks = k.narrow(0, kv_idx * self.kv_local * hd, self.kv_local * hd)
        vs = v.narrow(0, kv_idx * self.kv_local * hd, self.kv_local * hd)
        return torch.cat([qs, ks, vs], 0).contiguous()

    def full_shape(self, name):
        n = (self.heads + 2 * self.kv_heads) * self.head_dim
        return (n, self.weight.shape[1]) if name == "weight" else (n,)

    def forward(self, x, rms_eps=None):
        return ops.linear(x, self.weight, self.bias, rms_eps=rms_eps, w_scale=self.w_scale)


class GLUParallelLinear(_ShardLoadMixin, nn.Module):
    """Fused value/gate projection, rows interleaved (value_i, gate_i); output value*act(gate)."""

    def __init__(self, hidden: int, intermediate: int, act: str = "silu", bias: bool = False,
                 dtype=torch.bfloat16):
        super().__init__()
        st = tp()
        self.tp_rank, self.tp_size = st.rank, st.size
        self.act = act
        self.i_local = _div(intermediate, st.size)
        self.weight = nn.Parameter(torch.empty(2 * self.i_local, hidden, dtype=dtype), requires_grad=False)
        self.bias = nn.Parameter(torch.zeros(2 * self.i_local, dtype=dtype), requires_grad=False) if bias else None

    def _shard(self, name, full):
        return full.narrow(0, self.tp_rank * 2 * self.i_local, 2 * self.i_local).contiguous()

    def full_shape(self, name):
        n = 2 * self.i_local * self.tp_size
        return (n, self.weight.shape[1]) if name == "weight" else (n,)

    def forward(self, x, rms_eps=None):
        return ops.linear(x, self.weight, self.bias, act=self.act, glu=True, rms_eps=rms_eps, w_scale=self.w_scale)


class VocabParallelEmbedding(_ShardLoadMixin, nn.Module):
    def __init__(self, vocab: int, dim: int, dtype=torch.bfloat16):
        super().__init__()
        st = tp()
        self.tp_rank, self.tp_size = st.rank, st.size
        self.vocab = vocab
        self.v_local = (vocab + st.size - 1) // st.size
        self.start = self.tp_rank * self.v_local
        self.weight = nn.Parameter(torch.empty(self.v_local, dim, dtype=dtype), requires_grad=False)

    def _shard(self, name, full):
        out = torch.zeros(self.v_local, full.shape[1], dtype=full.dtype, device=full.device)
        n = max(0, min(self.v_local, self.vocab - self.start))
        out[:n] = full[self.start:self.start + n]
        return out

    def full_shape(self, name):
        return (self.vocab, self.weight.shape[1])

    def forward(self, ids):
        if self.tp_size == 1:
            return ops.embedding(ids, self.weight)
        local = ids - self.start
        valid = (local >= 0) & (local < self.v_local)
        y = ops.embedding(torch.where(valid, local, torch.zeros_like(local)), self.weight)
        y = y * valid.unsqueeze(-1).to(y.dtype)
        return comm.all_reduce(y.contiguous())


class ParallelLMHead(VocabParallelEmbedding):
    def logits(self, x, rms_eps=None):
        y = ops.linear(x, self.weight, rms_eps=rms_eps)
        if self.tp_size > 1:
            y = comm.all_gather_last(y)
        return y[..., : self.vocab]


FP8_LAYER_TYPES = (ColumnParallelLinear, RowParallelLinear, QKVParallelLinear, GLUParallelLinear)



@torch.no_grad()
def quantize_fp8_(model: nn.Module) -> int:
    """Quantise every TP linear layer of ``model`` to fp8 weights in place (embeddings / LM head
    stay bf16).  Call after any weight transform (e.g. RMSNorm gain folding).  Returns the count.
    A sub-module with ``no_fp8 = True`` (e.g. the mllama vision tower: vLLM's ``quantization: fp8`` leaves the
    vision encoder in bf16) keeps every linear under it bf16."""
    n = 0
    skip = set()
    for m in model.modules():
        if getattr(m, "no_fp8", False):
            skip.update(id(c) for c in m.modules())
    for m in model.modules():
        if isinstance(m, FP8_LAYER_TYPES) and id(m) not in skip:
            m.quantize_fp8_()
            n += 1
    return n
