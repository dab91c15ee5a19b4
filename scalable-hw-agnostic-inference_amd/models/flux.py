"""Flux.1 MMDiT transformer (black-forest-labs/FLUX.1-dev / -schnell), TP-aware.

Architecture (diffusers ``FluxTransformer2DModel``; the reference re-wraps it
for Neuron TP8 in app/src/transformer/model.py:143-447 and traces it in four
sub-graphs, app/src/transformer/compile.py:81-189):

* embedders: x_embedder (64 -> d), context_embedder (4096 -> d), and
  temb = TimestepEmbedding(t*1000) + TimestepEmbedding(guidance*1000) +
  PixArt text projection(pooled CLIP);
* 19 dual-stream blocks: AdaLN-Zero modulation (6 vectors per stream), joint
  attention over [text; image] with per-head RMSNorm on q/k and 3-axis RoPE,
  gated residual updates, GELU-tanh MLPs per stream;
* 38 single-stream blocks over the joint sequence: AdaLN-Zero (3 vectors),
  parallel attention + MLP whose outputs are concatenated into one proj_out;
* AdaLayerNormContinuous + proj_out (d -> 64).

MI355X design (not a translation of the reference's NxD wrappers):

* **Modulation hoisting** -- every AdaLN linear depends only on temb, i.e. on
  the timestep.  All 57+1 modulation GEMMs (3.2 B params) are evaluated ONCE
  per request for all denoising steps (M = steps x batch) instead of once per
  step as GEMVs: 6.4 GB of weight traffic per image instead of per step.
* **Joint-sequence layout without concat** -- the text/image QKV GEMMs write
  straight into the text/image rows of one packed [B, S, 3, H, D] buffer
  (strided GEMM output), so the joint attention reads it in place.
* **Fused epilogues** -- ``x += gate * (W h + b)`` is one GEMM epilogue
  (``ops.gemm_into(..., residual=x, gate=...)``, in place); GELU-tanh is fused
  into the MLP up-projection; LayerNorm + (1 + scale) / shift is one kernel
  (``ops.layernorm_mod``); RMSNorm(q), RMSNorm(k) and RoPE are one kernel
  (``ops.qk_norm_rope``) on the packed QKV buffer.
* **Single block proj_out as ONE GEMM + ONE all-reduce** at TP>1: the local
  columns [attention shard | MLP shard] of proj_out are gathered at load time,
  so the rank's concatenated [attn | mlp] activations feed a single GEMM (the
  reference splits it into two RowParallel layers and two all-reduces,
  app/src/transformer/model.py:303-322).
* **Sequence parallelism (optional, ``FluxConfig.sequence_parallel`` / ``SHAI_FLUX_SP=1``)** -- the
  reference disables SP (cova/mllama-32-11b-vllm-trn1-config.yaml:17) and runs Flux at TP8 only.  Here the
  38 single-stream blocks can keep the joint residual stream split into S/n-row shards over the TP group:
  LayerNorm-modulate and the gated residual run on S/n rows, an all-gather feeds the column-parallel
  QKV / MLP GEMMs and proj_out's partial sums are reduce-scattered instead of all-reduced (same bytes on
  xGMI as the all-reduce, 1/n of the norm / residual traffic and residual memory).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import torch
import torch.nn as nn

from .. import ops
from ..parallel import comm
from ..parallel.layers import ColumnParallelLinear, QKVParallelLinear, RowParallelLinear, _ShardLoadMixin
from ..parallel.state import tp
from .attention import merge_linear_keys
from .layers import BF16, Linear, timestep_embedding


@dataclass
class FluxConfig:
    in_channels: int = 64
    hidden: int = 3072
    heads: int = 24
    head_dim: int = 128
    num_layers: int = 19
    num_single_layers: int = 38
    mlp_ratio: float = 4.0
    joint_attention_dim: int = 4096
    pooled_projection_dim: int = 768
    guidance_embeds: bool = True
    axes_dims_rope: Tuple[int, int, int] = (16, 56, 56)
    rope_theta: float = 10000.0
    # Megatron-style sequence parallelism over the TP group for the single-stream blocks (SHAI_FLUX_SP=1)
    sequence_parallel: bool = field(default_factory=lambda: os.environ.get("SHAI_FLUX_SP", "0") == "1")

    @property
    def mlp_hidden(self) -> int:
        return int(self.hidden * self.mlp_ratio)

    @staticmethod
    def dev():
        return FluxConfig()

    @staticmethod
    def schnell():
        return FluxConfig(guidance_embeds=False)

    @staticmethod
    def tiny():
        return FluxConfig(hidden=128, heads=2, head_dim=64, num_layers=2, num_single_layers=2,
                          joint_attention_dim=64, pooled_projection_dim=32, axes_dims_rope=(16, 24, 24))


# ---------------------------------------------------------------------------- positional / time features
def rope_tables(ids: torch.Tensor, axes_dims: Sequence[int], theta: float) -> Tuple[torch.Tensor, torch.Tensor]:
    """FluxPosEmbed: ids [S, n_axes] -> cos/sin [S, sum(axes)/2] fp32 (one entry per rotation pair)."""
    cos, sin = [], []
    pos = ids.double()
    for i, d in enumerate(axes_dims):
        freqs = 1.0 / (theta ** (torch.arange(0, d, 2, dtype=torch.float64, device=ids.device) / d))
        ang = pos[:, i:i + 1] * freqs[None]
        cos.append(torch.cos(ang))
        sin.append(torch.sin(ang))
    return torch.cat(cos, -1).float().contiguous(), torch.cat(sin, -1).float().contiguous()


def latent_image_ids(h2: int, w2: int, device=None) -> torch.Tensor:
    ids = torch.zeros(h2, w2, 3, device=device)
    ids[..., 1] = torch.arange(h2, device=device)[:, None]
    ids[..., 2] = torch.arange(w2, device=device)[None, :]
    return ids.reshape(h2 * w2, 3)


def pack_latents(lat: torch.Tensor) -> torch.Tensor:
    """[B, C, h, w] -> [B, (h/2)(w/2), 4C] (2x2 patches, channel-major within a patch)."""
    B, C, h, w = lat.shape
    return lat.view(B, C, h // 2, 2, w // 2, 2).permute(0, 2, 4, 1, 3, 5).reshape(B, (h // 2) * (w // 2), C * 4)


def unpack_latents_nhwc(x: torch.Tensor, h: int, w: int) -> torch.Tensor:
    """[B, (h/2)(w/2), 4C] -> NHWC [B, h, w, C] (for the channels-last VAE)."""
    B, N, C4 = x.shape
    C = C4 // 4
    return x.view(B, h // 2, w // 2, C, 2, 2).permute(0, 1, 4, 2, 5, 3).reshape(B, h, w, C)


class MLPEmbedder(nn.Module):
    """linear_1 -> SiLU -> linear_2 (diffusers TimestepEmbedding / PixArtAlphaTextProjection)."""

    def __init__(self, din: int, d: int):
        super().__init__()
        self.linear_1 = Linear(din, d)
        self.linear_2 = Linear(d, d)

    def forward(self, x, residual=None):
        return self.linear_2(self.linear_1(x, act="silu"), residual=residual)


class TimeTextEmbed(nn.Module):
    def __init__(self, c: FluxConfig):
        super().__init__()
        self.timestep_embedder = MLPEmbedder(256, c.hidden)
        self.guidance_embedder = MLPEmbedder(256, c.hidden) if c.guidance_embeds else None
        self.text_embedder = MLPEmbedder(c.pooled_projection_dim, c.hidden)

    def forward(self, t: torch.Tensor, guidance: Optional[torch.Tensor], pooled: torch.Tensor) -> torch.Tensor:
        """t, guidance: [R] in [0, 1] (x1000 inside, as the reference wrapper, model.py:35-37); pooled [R, 768]."""
        dt = pooled.dtype
        e = self.timestep_embedder(timestep_embedding(t * 1000.0, 256, True, 0.0).to(dt))
        if self.guidance_embedder is not None and guidance is not None:
            e = self.guidance_embedder(timestep_embedding(guidance * 1000.0, 256, True, 0.0).to(dt), residual=e)
        return self.text_embedder(pooled, residual=e)


# ---------------------------------------------------------------------------- helpers
def _gated_out(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor], residual: torch.Tensor,
               gate: torch.Tensor, rows: int) -> None:
    """residual += gate[row // rows] * (x @ w^T + b), in place.  TP=1: one GEMM with the gated-residual epilogue;
    TP>1: partial GEMM -> all-reduce -> gated update (the gate multiplies the reduced sum)."""
    if tp().size == 1:
        ops.gemm_into(x, w, residual, b, residual=residual, gate=gate, rows_per_gate=rows)
        return
    # xGMI P2P: GEMM into the IPC staging slot (row slabs, each reduced beside the next slab's GEMM), then one kernel
    # per slab reduces and applies the gated residual in place
    nrows = x.numel() // x.shape[-1]
    if comm.row_parallel_reduce(x, w, b, residual, gate=gate, rows_per_gate=rows, out=residual,
                                chunks=comm.overlap_chunks(nrows, w.shape[0])) is not None:
        return
    y = ops.linear(x, w, None)
    comm.all_reduce(y)
    yb = y.float() + (b.float() if b is not None else 0.0)
    residual.add_((yb * gate.float().view(residual.shape[0], 1, -1)).to(residual.dtype))


def _gated_out_sp(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor], residual: torch.Tensor,
                  gate: torch.Tensor) -> None:
    """Sequence-parallel variant of :func:`_gated_out`: x is the full-sequence activation shard
    [B, S, in_local], residual this rank's sequence rows [B, S/n, d]; the partial GEMM output is
    reduce-scattered over the sequence, so the bias / gate / residual update touches S/n rows only."""
    y = comm.reduce_scatter_seq(ops.linear(x, w, None))
    yb = y.float() + (b.float() if b is not None else 0.0)
    residual.add_((yb * gate.float().view(residual.shape[0], 1, -1)).to(residual.dtype))


class _SingleProjOut(_ShardLoadMixin, nn.Module):
    """proj_out of a single-stream block: in = [attn (d) | mlp (mlp_hidden)] -> d.  At TP>1 the local
    input columns are [this rank's heads | this rank's MLP shard] so one GEMM + one all-reduce suffices."""

    def __init__(self, d: int, mlp_hidden: int):
        super().__init__()
        st = tp()
        self.rank, self.size, self.d, self.mlp = st.rank, st.size, d, mlp_hidden
        self.a_loc, self.m_loc = d // st.size, mlp_hidden // st.size
        self.weight = nn.Parameter(torch.empty(d, self.a_loc + self.m_loc, dtype=BF16), requires_grad=False)
        self.bias = nn.Parameter(torch.zeros(d, dtype=BF16), requires_grad=False)

    def _shard(self, name, full):
        if name == "bias":
            return full
        a = full[:, self.rank * self.a_loc:(self.rank + 1) * self.a_loc]
        m = full[:, self.d + self.rank * self.m_loc:self.d + (self.rank + 1) * self.m_loc]
        return torch.cat([a, m], 1).contiguous()

    def full_shape(self, name):
        return (self.d, self.d + self.mlp) if name == "weight" else (self.d,)


class FluxAttention(nn.Module):
    """Holds the fused projections and q/k RMSNorm weights of one block."""

    def __init__(self, c: FluxConfig, dual: bool):
        super().__init__()
        d, H, D = c.hidden, c.heads, c.head_dim
        self.qkv = QKVParallelLinear(d, H, H, D, bias=True)
        self.norm_q = nn.Parameter(torch.ones(D, dtype=BF16), requires_grad=False)
        self.norm_k = nn.Parameter(torch.ones(D, dtype=BF16), requires_grad=False)
        if dual:
            self.add_qkv = QKVParallelLinear(d, H, H, D, bias=True)
            self.norm_added_q = nn.Parameter(torch.ones(D, dtype=BF16), requires_grad=False)
            self.norm_added_k = nn.Parameter(torch.ones(D, dtype=BF16), requires_grad=False)
            self.to_out = RowParallelLinear(d, d)
            self.to_add_out = RowParallelLinear(d, d)


class FeedForward(nn.Module):
    def __init__(self, d: int, hidden: int):
        super().__init__()
        self.up = ColumnParallelLinear(d, hidden)
        self.down = RowParallelLinear(hidden, d)


class FluxTransformerBlock(nn.Module):
    def __init__(self, c: FluxConfig):
        super().__init__()
        d = c.hidden
        self.c = c
        self.norm1 = Linear(d, 6 * d)            # AdaLayerNormZero (image stream)
        self.norm1_context = Linear(d, 6 * d)    # AdaLayerNormZero (text stream)
        self.attn = FluxAttention(c, dual=True)
        self.ff = FeedForward(d, c.mlp_hidden)
        self.ff_context = FeedForward(d, c.mlp_hidden)

    def forward(self, img, txt, mod_img, mod_txt, cos, sin):
        """img [B, Ni, d], txt [B, Nt, d] updated in place; mod_* [B, 6d] (shift, scale, gate) x (msa, mlp)."""
        c = self.c
        B, Ni, d = img.shape
        Nt = txt.shape[1]
        S = Nt + Ni
        Hl = self.attn.qkv.h_local
        D = c.head_dim
        HD = Hl * D

        def chunk(m, i):
            return m[:, i * d:(i + 1) * d]

        xi = ops.layernorm_mod(img, chunk(mod_img, 1), chunk(mod_img, 0), Ni)
        xt = ops.layernorm_mod(txt, chunk(mod_txt, 1), chunk(mod_txt, 0), Nt)
        qkv = torch.empty(B, S, 3 * HD, dtype=img.dtype, device=img.device)
        ops.gemm_into(xt, self.attn.add_qkv.weight, qkv[:, :Nt], self.attn.add_qkv.bias)
        ops.gemm_into(xi, self.attn.qkv.weight, qkv[:, Nt:], self.attn.qkv.bias)
        for b in range(B):
            ops.qk_norm_rope(qkv[b, :Nt], self.attn.norm_added_q, self.attn.norm_added_k, cos[:Nt], sin[:Nt],
                             Hl, D, Nt)
            ops.qk_norm_rope(qkv[b, Nt:], self.attn.norm_q, self.attn.norm_k, cos[Nt:], sin[Nt:], Hl, D, Ni)
        q = qkv[..., :HD].view(B, S, Hl, D)
        k = qkv[..., HD:2 * HD].view(B, S, Hl, D)
        v = qkv[..., 2 * HD:].view(B, S, Hl, D)
        o = ops.attention(q, k, v).view(B, S, HD)
        _gated_out(o[:, Nt:], self.attn.to_out.weight, self.attn.to_out.bias, img, chunk(mod_img, 2), Ni)
        _gated_out(o[:, :Nt], self.attn.to_add_out.weight, self.attn.to_add_out.bias, txt, chunk(mod_txt, 2), Nt)
        # MLPs
        xi = ops.layernorm_mod(img, chunk(mod_img, 4), chunk(mod_img, 3), Ni)
        h = self.ff.up(xi, act="gelu_tanh")
        _gated_out(h, self.ff.down.weight, self.ff.down.bias, img, chunk(mod_img, 5), Ni)
        xt = ops.layernorm_mod(txt, chunk(mod_txt, 4), chunk(mod_txt, 3), Nt)
        h = self.ff_context.up(xt, act="gelu_tanh")
        _gated_out(h, self.ff_context.down.weight, self.ff_context.down.bias, txt, chunk(mod_txt, 5), Nt)


class FluxSingleTransformerBlock(nn.Module):
    def __init__(self, c: FluxConfig):
        super().__init__()
        d = c.hidden
        self.c = c
        self.norm = Linear(d, 3 * d)             # AdaLayerNormZeroSingle: shift, scale, gate
        self.attn = FluxAttention(c, dual=False)
        self.proj_mlp = ColumnParallelLinear(d, c.mlp_hidden)
        self.proj_out = _SingleProjOut(d, c.mlp_hidden)

    def forward(self, x, mod, cos, sin, sp: bool = False):
        """x [B, S, d] joint sequence, updated in place; mod [B, 3d].  sp: x holds only this rank's S/n
        sequence rows (sequence parallel): the normalised rows are all-gathered before the column-parallel
        QKV / MLP GEMMs and proj_out's partial sums are reduce-scattered back onto the local rows."""
        c = self.c
        B, s_loc, d = x.shape
        Hl = self.attn.qkv.h_local
        D = c.head_dim
        HD = Hl * D
        xn = ops.layernorm_mod(x, mod[:, d:2 * d], mod[:, :d], s_loc)
        S = s_loc * tp().size if sp else s_loc
        qkv = torch.empty(B, S, 3 * HD, dtype=x.dtype, device=x.device)
        cat = torch.empty(B, S, HD + self.proj_mlp.out_local, dtype=x.dtype, device=x.device)
        specs = [(self.attn.qkv.weight, self.attn.qkv.bias, None, qkv),
                 (self.proj_mlp.weight, self.proj_mlp.bias, "gelu_tanh", cat[..., HD:])]
        if sp:   # the sequence all-gather forked beside this rank's own rows' GEMMs (comm.gather_seq_linears)
            comm.gather_seq_linears(xn, specs)
        else:
            for w, b, act, out in specs:
                ops.gemm_into(xn, w, out, b, act=act)
        ops.qk_norm_rope(qkv.view(B * S, 3 * HD), self.attn.norm_q, self.attn.norm_k, cos, sin, Hl, D, S)
        ops.attention(qkv[..., :HD].view(B, S, Hl, D), qkv[..., HD:2 * HD].view(B, S, Hl, D),
                      qkv[..., 2 * HD:].view(B, S, Hl, D), out=cat[..., :HD].view(B, S, Hl, D))
        if sp:
            _gated_out_sp(cat, self.proj_out.weight, self.proj_out.bias, x, mod[:, 2 * d:])
        else:
            _gated_out(cat, self.proj_out.weight, self.proj_out.bias, x, mod[:, 2 * d:], S)


class FluxTransformer2DModel(nn.Module):
    def __init__(self, cfg: FluxConfig = None):
        super().__init__()
        self.cfg = c = cfg or FluxConfig()
        assert sum(c.axes_dims_rope) == c.head_dim
        self.x_embedder = Linear(c.in_channels, c.hidden)
        self.context_embedder = Linear(c.joint_attention_dim, c.hidden)
        self.time_text_embed = TimeTextEmbed(c)
        self.transformer_blocks = nn.ModuleList([FluxTransformerBlock(c) for _ in range(c.num_layers)])
        self.single_transformer_blocks = nn.ModuleList([FluxSingleTransformerBlock(c)
                                                        for _ in range(c.num_single_layers)])
        self.norm_out = Linear(c.hidden, 2 * c.hidden)   # AdaLayerNormContinuous: scale, shift
        self.proj_out = Linear(c.hidden, c.in_channels)

    # -------------------------------------------------------------- per-request precompute
    def mod_layout(self) -> Tuple[List[Tuple[int, int]], List[int], int, int]:
        """Column offsets of every block's modulation vectors inside one [R, total] tensor:
        dual (img, txt) offsets (6d each), single offsets (3d each), norm_out offset (2d), total."""
        d = self.cfg.hidden
        off, dual, single = 0, [], []
        for _ in self.transformer_blocks:
            dual.append((off, off + 6 * d))
            off += 12 * d
        for _ in self.single_transformer_blocks:
            single.append(off)
            off += 3 * d
        return dual, single, off, off + 2 * d

    @torch.no_grad()
    def modulations(self, t: torch.Tensor, guidance: Optional[torch.Tensor], pooled: torch.Tensor) -> torch.Tensor:
        """All AdaLN modulation vectors for R = steps x batch rows (t / guidance / pooled per row) in ONE
        [R, total] tensor (layout: :meth:`mod_layout`), each block's linear run once with M = R."""
        temb = self.time_text_embed(t, guidance, pooled)
        st = ops.bias_act(temb, None, None, act="silu")
        dual, single, o_out, total = self.mod_layout()
        d = self.cfg.hidden
        out = torch.empty(st.shape[0], total, dtype=st.dtype, device=st.device)
        for blk, (oi, ot) in zip(self.transformer_blocks, dual):
            ops.gemm_into(st, blk.norm1.weight, out[:, oi:oi + 6 * d], blk.norm1.bias)
            ops.gemm_into(st, blk.norm1_context.weight, out[:, ot:ot + 6 * d], blk.norm1_context.bias)
        for blk, o in zip(self.single_transformer_blocks, single):
            ops.gemm_into(st, blk.norm.weight, out[:, o:o + 3 * d], blk.norm.bias)
        ops.gemm_into(st, self.norm_out.weight, out[:, o_out:], self.norm_out.bias)
        return out

    def rope(self, txt_len: int, h2: int, w2: int, device) -> Tuple[torch.Tensor, torch.Tensor]:
        ids = torch.cat([torch.zeros(txt_len, 3, device=device), latent_image_ids(h2, w2, device)], 0)
        return rope_tables(ids, self.cfg.axes_dims_rope, self.cfg.rope_theta)

    @torch.no_grad()
    def forward_step(self, latents: torch.Tensor, ctx: torch.Tensor, mod: torch.Tensor, cos, sin) -> torch.Tensor:
        """One denoising step.  latents [B, Ni, 64] packed; ctx = context_embedder(T5 states) [B, Nt, d]
        (step invariant, computed once per request); mod [B, total]: this step's rows of modulations().
        Returns the flow (velocity) prediction [B, Ni, 64]."""
        B, Ni, _ = latents.shape
        Nt = ctx.shape[1]
        d = self.cfg.hidden
        dual, single, o_out, _ = self.mod_layout()
        img = self.x_embedder(latents)
        joint = torch.empty(B, Nt + Ni, d, dtype=img.dtype, device=img.device)
        joint[:, :Nt].copy_(ctx)
        joint[:, Nt:].copy_(img)
        txt, img = joint[:, :Nt], joint[:, Nt:]
        for blk, (oi, ot) in zip(self.transformer_blocks, dual):
            blk(img, txt, mod[:, oi:oi + 6 * d], mod[:, ot:ot + 6 * d], cos, sin)
        st = tp()
        if self.cfg.sequence_parallel and st.size > 1 and (Nt + Ni) % st.size == 0:
            # SP over the TP group: the joint residual stream is split into S/n-row shards for the single
            # blocks (replicated after the dual blocks, so slicing needs no communication)
            s = (Nt + Ni) // st.size
            xs = joint[:, st.rank * s:(st.rank + 1) * s].contiguous()
            for blk, o in zip(self.single_transformer_blocks, single):
                blk(xs, mod[:, o:o + 3 * d], cos, sin, sp=True)
            joint = comm.all_gather_seq(xs)
        else:
            for blk, o in zip(self.single_transformer_blocks, single):
                blk(joint, mod[:, o:o + 3 * d], cos, sin)
        mo = mod[:, o_out:]
        x = ops.layernorm_mod(joint[:, Nt:], mo[:, :d], mo[:, d:], Ni)
        return self.proj_out(x)

    def forward(self, latents, encoder_hidden_states, pooled, timestep, guidance=None, img_hw=None):
        """Convenience single call (tests): latents [B, Ni, 64], T5 states [B, Nt, 4096], pooled [B, 768],
        timestep / guidance [B] in [0, 1]; img_hw = (h/2, w/2) of the packed latent grid."""
        B, Ni, _ = latents.shape
        Nt = encoder_hidden_states.shape[1]
        h2, w2 = img_hw or (int(math.isqrt(Ni)), Ni // int(math.isqrt(Ni)))
        mod = self.modulations(timestep, guidance, pooled)
        cos, sin = self.rope(Nt, h2, w2, latents.device)
        ctx = self.context_embedder(encoder_hidden_states)
        return self.forward_step(latents, ctx, mod, cos, sin)

    # -------------------------------------------------------------- checkpoints
    def convert_hf_state_dict(self, sd: dict) -> dict:
        """diffusers FluxTransformer2DModel keys -> this module (fused q/k/v, renamed FF / norms)."""
        out = {}
        for k, v in sd.items():
            k2 = k.replace(".ff.net.0.proj.", ".ff.up.").replace(".ff.net.2.", ".ff.down.")
            k2 = k2.replace(".ff_context.net.0.proj.", ".ff_context.up.").replace(".ff_context.net.2.",
                                                                                  ".ff_context.down.")
            k2 = k2.replace(".attn.to_out.0.", ".attn.to_out.").replace(".norm1.linear.", ".norm1.")
            k2 = k2.replace(".norm1_context.linear.", ".norm1_context.").replace(".norm.linear.", ".norm.")
            k2 = k2.replace("norm_out.linear.", "norm_out.")
            for n in ("norm_q", "norm_k", "norm_added_q", "norm_added_k"):
                k2 = k2.replace(f".attn.{n}.weight", f".attn.{n}")
            out[k2] = v
        for i in range(self.cfg.num_layers):
            p = f"transformer_blocks.{i}.attn."
            merge_linear_keys(out, p, ["to_q", "to_k", "to_v"], "qkv")
            merge_linear_keys(out, p, ["add_q_proj", "add_k_proj", "add_v_proj"], "add_qkv")
        for i in range(self.cfg.num_single_layers):
            merge_linear_keys(out, f"single_transformer_blocks.{i}.attn.", ["to_q", "to_k", "to_v"], "qkv")
        return out
