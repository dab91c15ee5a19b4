"""Operator layer: thin wrappers over the gfx950 HIP kernels (``torch.ops.shai``).

GPU tensors always go to the native kernels (raising if the library is not
built -- no silent eager fallback).  CPU tensors use the fp32 references in
:mod:`shai_amd.ops.reference` (tests / CPU plumbing config).

All wrappers allocate their outputs with torch (graph-pool aware), launch on
the current stream and never synchronise, so whole model steps can be
captured into HIP graphs (``torch.cuda.CUDAGraph`` is hipGraph on ROCm).
"""
from __future__ import annotations

import math
import os
from typing import Optional, Tuple

import torch

from .. import native
from . import reference as ref
from .reference import (ACT_GELU, ACT_GELU_TANH, ACT_NONE, ACT_QUICK_GELU, ACT_RELU, ACT_SILU, act_id,
                        pack_conv_weight, pack_up2_phase_weight, unpack_conv_weight)

__all__ = [
    "rmsnorm", "layernorm", "groupnorm_stats", "groupnorm_apply", "groupnorm", "linear", "conv2d", "attention",
    "paged_attention", "decode_attention", "kv_write", "rope", "rope_pairs", "gated_act", "bias_act", "sched_step",
    "softmax_", "embedding", "token_feedback", "decode_attention_rope", "decode_attention_rope_qkv", "gemm_partials", "quantize_fp8_rows", "dequant_fp8", "quant_rows_fp8", "gemm_f8", "pack_conv_weight", "pack_up2_phase_weight", "linear_wslices", "unpack_conv_weight", "act_id", "ACT_NONE", "ACT_SILU", "ACT_GELU",
    "ACT_GELU_TANH", "ACT_QUICK_GELU", "ACT_RELU", "decode_splits", "set_decode_wb",
]


def _gpu(t: torch.Tensor) -> bool:
    return t.is_cuda


def _K():
    return native.ops()


def _i32(t: Optional[torch.Tensor]):
    if t is None:
        return None
    return t if t.dtype == torch.int32 else t.to(torch.int32)


# ----------------------------------------------------------------------------- norms
def rmsnorm(x: torch.Tensor, w: Optional[torch.Tensor], eps: float = 1e-6, residual: Optional[torch.Tensor] = None,
            w_offset: float = 0.0, out: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """y = rmsnorm(x (+ residual)) * (w + w_offset); returns (y, x + residual or None)."""
    if not _gpu(x):
        return ref.rmsnorm(x, w, eps, residual, w_offset)
    shape = x.shape
    x2 = x if x.dim() == 2 else x.reshape(-1, shape[-1])
    res2 = residual.reshape(-1, shape[-1]) if residual is not None else None
    y = out if out is not None else torch.empty(x2.shape, dtype=x.dtype, device=x.device)
    new_res = torch.empty(x2.shape, dtype=x.dtype, device=x.device) if residual is not None else None
    _K().rmsnorm(x2, w, y, res2, new_res, float(eps), float(w_offset))
    return y.view(shape), (new_res.view(shape) if new_res is not None else None)


def layernorm(x: torch.Tensor, w: Optional[torch.Tensor], b: Optional[torch.Tensor], eps: float = 1e-5,
              residual: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    if not _gpu(x):
        return ref.layernorm(x, w, b, eps, residual)
    shape = x.shape
    x2 = x if x.dim() == 2 else x.reshape(-1, shape[-1])
    res2 = residual.reshape(-1, shape[-1]) if residual is not None else None
    y = torch.empty(x2.shape, dtype=x.dtype, device=x.device)
    new_res = torch.empty(x2.shape, dtype=x.dtype, device=x.device) if residual is not None else None
    _K().layernorm(x2, w, b, y, res2, new_res, float(eps))
    return y.view(shape), (new_res.view(shape) if new_res is not None else None)


_GN_TICKETS: dict = {}
# Finalize fused into the stats launch (last-block ticket) is opt-in: on MI355X the per-block
# agent-scope add + vmcnt drain made GN+SiLU 1.3-1.45x SLOWER than a separate 8-block finalize
# launch (8x4096x320: 40.6 vs 28.2 us), so the two-launch path stays the default.
_GN_FUSED = os.environ.get("SHAI_GN_FUSED_FINALIZE", "0") == "1"


def _gn_tickets(x: torch.Tensor, n: int) -> Optional[torch.Tensor]:
    """Zeroed int32 tickets for the stats kernel's fused finalize, one set per (device, stream):
    the kernel re-arms them to 0, so they stay valid across launches and HIP-graph replays."""
    if not _GN_FUSED or n > 4096:
        return None
    key = (x.device.index, torch.cuda.current_stream(x.device).cuda_stream)
    t = _GN_TICKETS.get(key)
    if t is None:
        t = _GN_TICKETS[key] = torch.zeros(4096, dtype=torch.int32, device=x.device)
    return t


def _scale_shift_pair(n: int, c: int, device):
    """GroupNorm (scale, shift) [n, c] fp32 as the two halves of ONE allocation (shift = scale + n c): the layout
    the halo-tiled conv's scale / shift DMA reads (csrc/kernels/conv_halo.hip)."""
    ss = torch.empty(2, n, c, dtype=torch.float32, device=device)
    return ss[0], ss[1]


def groupnorm_stats(x: torch.Tensor, gamma, beta, groups: int, eps: float, x2: Optional[torch.Tensor] = None):
    """Channels-last GroupNorm statistics. x [N, ..., C] -> (scale, shift) fp32 [N, C].
    With ``x2`` the statistics are those of ``cat([x, x2], -1)`` without materialising it."""
    N = x.shape[0]
    x3 = x.reshape(N, -1, x.shape[-1])
    x23 = x2.reshape(N, -1, x2.shape[-1]) if x2 is not None else None
    C = x3.shape[-1] + (x23.shape[-1] if x23 is not None else 0)
    if not _gpu(x):
        xx = torch.cat([x3, x23], -1) if x23 is not None else x3
        return ref.groupnorm_stats(xx, gamma, beta, groups, eps)
    part = torch.empty(N * 256 * groups * 2, dtype=torch.float32, device=x.device)
    scale, shift = _scale_shift_pair(N, C, x.device)
    _K().groupnorm_stats(x3, x23, gamma, beta, part, scale, shift, _gn_tickets(x, N), int(groups), float(eps))
    return scale, shift


def groupnorm_apply(x: torch.Tensor, scale, shift, silu: bool = False, x2: Optional[torch.Tensor] = None) -> torch.Tensor:
    """y = (silu)(x * scale + shift); with ``x2`` the input is ``cat([x, x2], -1)`` (never materialised)."""
    if not _gpu(x):
        xx = torch.cat([x, x2], -1) if x2 is not None else x
        return ref.groupnorm_apply(xx, scale, shift, silu)
    N = x.shape[0]
    C = x.shape[-1] + (x2.shape[-1] if x2 is not None else 0)
    out = torch.empty(*x.shape[:-1], C, dtype=x.dtype, device=x.device)
    _K().groupnorm_apply(x.reshape(N, -1, x.shape[-1]), x2.reshape(N, -1, x2.shape[-1]) if x2 is not None else None,
                         scale, shift, out.view(N, -1, C), bool(silu))
    return out


def groupnorm(x, gamma, beta, groups, eps, silu=False, x2=None):
    scale, shift = groupnorm_stats(x, gamma, beta, groups, eps, x2=x2)
    return groupnorm_apply(x, scale, shift, silu, x2=x2)


# ----------------------------------------------------------------------------- GEMM / conv
FP8_E4M3_MAX = 448.0


def quantize_fp8_rows(w: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """Per-output-row symmetric fp8 (OCP e4m3) quantisation: w ~= w8 * scale[:, None].
    One-time load transform (not a hot op): returns (w8 float8_e4m3fn [N, K], scale fp32 [N])."""
    wf = w.float()
    scale = (wf.abs().amax(dim=1) / FP8_E4M3_MAX).clamp(min=1e-12)
    w8 = (wf / scale[:, None]).clamp(-FP8_E4M3_MAX, FP8_E4M3_MAX).to(torch.float8_e4m3fn)
    return w8.contiguous(), scale.contiguous()


def dequant_fp8(w8: torch.Tensor, scale: torch.Tensor, dtype=torch.bfloat16) -> torch.Tensor:
    """w8 * scale[:, None] -> bf16 (native kernel on the GPU)."""
    if not w8.is_cuda:
        return (w8.float() * scale.float()[:, None]).to(dtype)
    out = torch.empty(w8.shape, dtype=torch.bfloat16, device=w8.device)
    _K().dequant_fp8(w8, scale, out)
    return out


# fp8 weights on problems of more than 64 rows (prefill): "w8a8" quantises the activation per row on the fly and
# runs the fp8 MFMA GEMM (gemm_f8.hip); "dequant" widens the weights to bf16 and runs the bf16 GEMMs
FP8_PREFILL = os.environ.get("SHAI_FP8_PREFILL", "w8a8")


def quant_rows_fp8(x: torch.Tensor, rms_eps: Optional[float] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Per-row e4m3 quantisation of a 2-D bf16 activation: x ~= a8 * scale[:, None] (scale = absmax / 448).
    With ``rms_eps`` the row's RMSNorm rstd is multiplied into the scale (the consumer's weights carry the
    folded norm gain), so the product a8 @ w^T * scale is the product of the normalised row."""
    if not _gpu(x):
        return ref.quant_rows_fp8(x, rms_eps)
    M, K = x.shape
    a8 = torch.empty(M, K, dtype=torch.float8_e4m3fn, device=x.device)
    scale = torch.empty(M, dtype=torch.float32, device=x.device)
    _K().quant_rows_fp8(x, a8, scale, float(rms_eps) if rms_eps is not None else -1.0)
    return a8, scale


def gemm_f8(a8: torch.Tensor, w8: torch.Tensor, a_scale: torch.Tensor, w_scale: torch.Tensor,
            bias: Optional[torch.Tensor] = None, act=None, residual: Optional[torch.Tensor] = None,
            glu: bool = False, res_alpha: float = 1.0, cfg: int = -1,
            out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """W8A8 GEMM on the fp8 MFMA: act(a_scale[m] * w_scale[n] * a8 @ w8^T + bias) (+ res_alpha * residual),
    GLU as in ``linear``; bf16 output."""
    if not _gpu(a8):
        return ref.gemm_f8(a8, w8, a_scale, w_scale, bias, act, residual, glu, res_alpha)
    N = w8.shape[0]
    y = out if out is not None else torch.empty(a8.shape[0], N // 2 if glu else N, dtype=torch.bfloat16,
                                                device=a8.device)
    _K().gemm_f8(a8, w8, a_scale, w_scale, y, bias, residual, float(res_alpha), act_id(act), bool(glu), int(cfg))
    return y


def linear(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None, act=None,
           residual: Optional[torch.Tensor] = None, glu: bool = False, alpha: float = 1.0,
           res_alpha: float = 1.0, rms_eps: Optional[float] = None,
           w_scale: Optional[torch.Tensor] = None, row_affine=None, force_cfg: int = -1) -> torch.Tensor:
    """y = act(alpha * x @ w^T + bias) (+ res_alpha * residual).

    glu=True: ``w`` rows are interleaved (value_i, gate_i) pairs and the output
    has N/2 columns: value * act(gate) (SwiGLU / GEGLU fused in the epilogue).
    rms_eps: x is RMS-normalised first (unweighted: the norm gain must already be
    folded into w's columns); on the GPU this is fused into the decode GEMM.
    row_affine = (mr [M, 2] fp32, s [N] fp32): a LayerNorm of x folded into the GEMM -- y = rstd[m] * (x @ w^T -
    mean[m] * s[n]) + bias, with the norm gain / shift pre-folded into w / bias (``fold_layernorm``) and
    (mean, rstd) from the producer of x (``linear_stats`` / ``conv2d(stats="ln")``).
    w_scale: ``w`` is fp8 e4m3 with one fp32 scale per row (``quantize_fp8_rows``).  Decode-shaped
    problems (<= 64 rows) stream the fp8 bytes through the skinny kernel (half the weight
    traffic); larger ones run W8A8 on the fp8 MFMA (``FP8_PREFILL``: the activation is quantised per row, with
    the folded RMSNorm in its row scale) or dequantize to bf16 first and run the bf16 GEMMs.
    """
    if w_scale is not None:
        M = x.numel() // x.shape[-1]
        K = x.shape[-1]
        if (_gpu(x) and M > 64 and FP8_PREFILL == "w8a8" and alpha == 1.0 and K % 16 == 0
                and (not glu or w.shape[0] % 4 == 0)):
            x2 = x.reshape(-1, K) if (x.dim() == 2 or x.is_contiguous()) else x.contiguous().reshape(-1, K)
            a8, a_scale = quant_rows_fp8(x2, rms_eps)
            N = w.shape[0] // 2 if glu else w.shape[0]
            r2 = residual.reshape(-1, N) if residual is not None else None
            y = gemm_f8(a8, w, a_scale, w_scale, bias, act, r2, glu, res_alpha)
            return y.view(*x.shape[:-1], N)
        if not _gpu(x) or M > 64 or K % 16 != 0:
            w = dequant_fp8(w, w_scale)
            w_scale = None
    if not _gpu(x):
        if rms_eps is not None:
            x = ref.rmsnorm(x, None, rms_eps)[0]
        return ref.linear(x, w, bias, act, residual, glu, alpha, res_alpha, row_affine=row_affine)
    if row_affine is not None:
        return _linear_norm_io(x, w, bias, act, residual, glu, alpha, res_alpha, row_affine, None, 0.0, force_cfg)[0]
    K = x.shape[-1]
    N = w.shape[0]
    lead = x.shape[:-1]
    if x.dim() == 2 or x.is_contiguous():
        x2 = x.reshape(-1, K)
    else:
        x2 = x.contiguous().reshape(-1, K)
    Nout = N // 2 if glu else N
    y = torch.empty(x2.shape[0], Nout, dtype=x.dtype, device=x.device)
    r2 = residual.reshape(-1, Nout) if residual is not None else None
    _K().gemm(x2, w, y, bias, None, 1, r2, float(alpha), float(res_alpha), act_id(act), bool(glu), None, 1, -1,
              float(rms_eps) if rms_eps is not None else -1.0, w_scale)
    return y.view(*lead, Nout)


def _linear_norm_io(x, w, bias, act, residual, glu, alpha, res_alpha, row_affine, stats, eps, force_cfg=-1):
    K = x.shape[-1]
    x2 = x.reshape(-1, K) if (x.dim() == 2 or x.is_contiguous()) else x.contiguous().reshape(-1, K)
    M, N = x2.shape[0], w.shape[0]
    Nout = N // 2 if glu else N
    y = torch.empty(M, Nout, dtype=x.dtype, device=x.device)
    r2 = residual.reshape(-1, Nout) if residual is not None else None
    mr, s = row_affine if row_affine is not None else (None, None)
    gp = torch.empty(M // 128, Nout, 2, dtype=torch.float32, device=x.device) if stats == "gn" else None
    ls = torch.empty(M, 2, dtype=torch.float32, device=x.device) if stats == "ln" else None
    _K().gemm(x2, w, y, bias, None, 1, r2, float(alpha), float(res_alpha), act_id(act), bool(glu), None, 1,
              int(force_cfg), -1.0, None, mr, s, gp, ls, float(eps))
    return y.view(*x.shape[:-1], Nout), (gp if stats == "gn" else ls)


def stats_supported(rows: int, cols: int, kind: str, hw: Optional[int] = None) -> bool:
    """Whether ``linear_stats`` / ``conv2d(stats=...)`` can hand statistics of this output to the next norm:
    GroupNorm partials need 128-row blocks inside one image (hw % 128 == 0), N % 8 == 0, N <= 2048."""
    if cols % 8 != 0:
        return False
    if kind == "gn":
        return rows % 128 == 0 and cols <= 2048 and (hw is None or hw % 128 == 0)
    return True


def fold_profitable(rows: int, cols: int) -> bool:
    """A LayerNorm folded into a GEMM pins that GEMM to the v4 kernel (256-row tiles, unsplit): worth it only when
    the problem has about a wave of 256 x 320 tiles for the 256 CUs -- otherwise the standalone norm pass plus the
    tuner's choice (smaller tiles, split-K) is faster (SD2.1 at batch 1: 32 tiles)."""
    return ((rows + 255) // 256) * ((cols + 319) // 320) >= FOLD_MIN_TILES


FOLD_MIN_TILES = int(os.environ.get("SHAI_FOLD_MIN_TILES", "192"))  # tests lower it to force the folded path


def linear_stats(x: torch.Tensor, w: torch.Tensor, bias=None, residual=None, act=None, stats: str = "ln",
                 eps: float = 1e-5, row_affine=None, force_cfg: int = -1):
    """``linear`` that also returns statistics of its output for the next norm: stats="ln" -> (mean, rstd) [M, 2]
    with ``eps``; "gn" -> GroupNorm partials [M / 128, N, 2] (``groupnorm_stats_from_partials``).  On the GPU the
    v4 GEMM epilogue writes them (a pass over the output when the tuned kernel cannot)."""
    if not _gpu(x):
        y = ref.linear(x, w, bias, act, residual, False, 1.0, 1.0, row_affine=row_affine)
        y2 = y.reshape(-1, y.shape[-1])
        return y, (ref.row_moments(y2, eps) if stats == "ln" else ref.col_partials(y2))
    return _linear_norm_io(x, w, bias, act, residual, False, 1.0, 1.0, row_affine, stats, eps, force_cfg)


def linear_wslices(x: torch.Tensor, w_slices: torch.Tensor, bias2d: Optional[torch.Tensor], rows_per_slice: int,
                   stats: Optional[str] = None, eps: float = 1e-5):
    """y[rows of slice s] = x[rows] w_slices[s]^T + bias2d[s]: one GEMM whose row blocks of ``rows_per_slice`` rows
    (multiples of 256) each take their own weight [N, K] -- e.g. a GroupNorm's per-image scale folded into the
    following projection's weight (``Transformer2DModel``).  x [M, K], w_slices [M / rows_per_slice, N, K], bias2d
    [M / rows_per_slice, N].  ``stats`` as ``linear_stats`` (returns (y, st) then)."""
    S, N, K = w_slices.shape
    M = x.shape[0]
    if not _gpu(x):
        y = torch.einsum("smk,snk->smn", x.float().view(S, M // S, K), w_slices.float())
        if bias2d is not None:
            y = y + bias2d.float()[:, None, :]
        y = y.reshape(M, N).to(x.dtype)
        if stats is None:
            return y
        return y, (ref.row_moments(y, eps) if stats == "ln" else ref.col_partials(y))
    y = torch.empty(M, N, dtype=x.dtype, device=x.device)
    gp = torch.empty(M // 128, N, 2, dtype=torch.float32, device=x.device) if stats == "gn" else None
    ls = torch.empty(M, 2, dtype=torch.float32, device=x.device) if stats == "ln" else None
    _K().gemm(x, w_slices.reshape(S * N, K), y, None, bias2d, int(rows_per_slice), None, 1.0, 1.0, ACT_NONE, False,
              None, 1, -1, -1.0, None, None, None, gp, ls, float(eps), int(rows_per_slice))
    if stats is None:
        return y
    return y, (gp if stats == "gn" else ls)


def linear_lnout(x: torch.Tensor, w: torch.Tensor, bias, residual: torch.Tensor, gamma, beta, eps: float = 1e-5):
    """(y, LayerNorm(y; gamma, beta)) with y = x @ w^T + bias + residual: the next LayerNorm computed by the producing
    GEMM's epilogue (the W-stationary kernel holds whole 320-wide rows: exact two-pass moments of the stored bf16 y),
    so the consumer runs a plain GEMM on the normalised rows.  Falls back to GEMM + standalone LayerNorm wherever
    the fused kernel does not apply (other widths, CPU)."""
    if not _gpu(x):
        y = ref.linear(x, w, bias, None, residual)
        return y, ref.layernorm(y, gamma, beta, eps)[0]
    K, N = x.shape[-1], w.shape[0]
    x2 = x.reshape(-1, K) if (x.dim() == 2 or x.is_contiguous()) else x.contiguous().reshape(-1, K)
    r2 = residual.reshape(-1, N)
    y = torch.empty(x2.shape[0], N, dtype=x.dtype, device=x.device)
    y2 = torch.empty_like(y)
    if LNOUT and _K().gemm_lnout(x2, w, y, y2, bias, r2, 1.0, gamma, beta, float(eps)):
        return y.view(*x.shape[:-1], N), y2.view(*x.shape[:-1], N)
    y = linear(x, w, bias, residual=residual)
    return y, layernorm(y, gamma, beta, eps)[0]


LNOUT = os.environ.get("SHAI_LNOUT", "1") != "0"  # A/B switch for the producer-side LayerNorm (linear_lnout)


def lnout_supported(rows: int, n: int, k: int) -> bool:
    """Whether linear_lnout runs fused on the GPU (W-stationary kernel: K = N = 320)."""
    return LNOUT and n == 320 and k == 320


def fold_layernorm(w: torch.Tensor, bias: Optional[torch.Tensor], gamma: Optional[torch.Tensor],
                   beta: Optional[torch.Tensor]):
    """(w', bias', s) so that LayerNorm(x; gamma, beta) @ w^T + bias == rstd * (x @ w'^T - mean * s) + bias':
    w' = w * gamma (columns), bias' = bias + w @ beta, s = row sums of w' (fp32, from its bf16 values)."""
    wf = w.float()
    w2 = (wf * gamma.float()[None, :]).to(w.dtype) if gamma is not None else w
    b2 = bias.float() if bias is not None else torch.zeros(w.shape[0], dtype=torch.float32, device=w.device)
    if beta is not None:
        b2 = b2 + wf @ beta.float()
    return w2.contiguous(), b2.to(w.dtype), w2.float().sum(1).contiguous()


def row_moments(x: torch.Tensor, eps: float) -> torch.Tensor:
    """(mean, rstd) [M, 2] of the rows of x [..., N] (the statistics a folded LayerNorm consumes)."""
    x2 = x.reshape(-1, x.shape[-1])
    if not _gpu(x):
        return ref.row_moments(x2, eps)
    mr = torch.empty(x2.shape[0], 2, dtype=torch.float32, device=x.device)
    _K().row_moments(x2, mr, float(eps))
    return mr


def col_partials(x: torch.Tensor) -> torch.Tensor:
    """GroupNorm partials [M / 128, N, 2] of x [..., N] (rows grouped by 128)."""
    x2 = x.reshape(-1, x.shape[-1])
    if not _gpu(x):
        return ref.col_partials(x2)
    part = torch.empty(x2.shape[0] // 128, x2.shape[1], 2, dtype=torch.float32, device=x.device)
    _K().col_partials(x2, part)
    return part


def groupnorm_stats_from_partials(part: torch.Tensor, gamma, beta, groups: int, eps: float, nimg: int, hw: int,
                                  part2: Optional[torch.Tensor] = None):
    """GroupNorm (scale, shift) fp32 [N, C] from the partials of x (and of x2 for cat([x, x2], -1))."""
    C1 = part.shape[-2]
    C2 = part2.shape[-2] if part2 is not None else 0
    if not part.is_cuda:
        return ref.groupnorm_from_partials(part, part2, C1, C2, nimg, hw, gamma, beta, groups, eps)
    scale, shift = _scale_shift_pair(nimg, C1 + C2, part.device)
    _K().groupnorm_from_partials(part, part2, C1, C2, nimg, hw, gamma, beta, scale, shift, int(groups), float(eps))
    return scale, shift


def gemm_into(x: torch.Tensor, w: torch.Tensor, out: torch.Tensor, bias=None, act=None, residual=None, gate=None,
              rows_per_gate: int = 1, alpha: float = 1.0, res_alpha: float = 1.0, glu: bool = False,
              force_cfg: int = -1, rms_eps: float = -1.0, w_scale: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out = gate[row // rows_per_gate] * act(alpha * x @ w^T + bias) + res_alpha * residual, written into ``out``.
    rms_eps >= 0: x is RMS-normalised first (unweighted; fold the gain into w).
    w_scale: fp8 e4m3 ``w`` with per-row scales (skinny kernel only, as in ``linear``).
    force_cfg (tests / tools): a tile config index, 1000 (+ kg) = skinny kernel with a separate split-K fold,
    1100 + kg = skinny kernel reducing its K groups inside the launch, 2000 = hipBLASLt.

    x / out / residual are 2D [M, *] or 3D [B, M, *] views whose rows may be strided
    (e.g. the text / image halves of a joint-sequence buffer); the row index used
    for ``gate`` is the flattened b * M + m (AdaLN-Zero gates per image)."""
    if not _gpu(x):
        if w_scale is not None:
            w = dequant_fp8(w, w_scale)
        if rms_eps >= 0:
            x = ref.rmsnorm(x, None, rms_eps)[0]
        return ref.gemm_into(x, w, out, bias, act, residual, gate, rows_per_gate, alpha, res_alpha, glu)
    _K().gemm(x, w, out, bias, None, 1, residual, float(alpha), float(res_alpha), act_id(act), bool(glu), gate,
              int(rows_per_gate), int(force_cfg), float(rms_eps), w_scale)
    return out


def layernorm_mod(x: torch.Tensor, scale: torch.Tensor, shift: torch.Tensor, rows_per_mod: int,
                  eps: float = 1e-6, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """AdaLN: LayerNorm(x) (no affine) * (1 + scale[r // rows_per_mod]) + shift[r // rows_per_mod].
    scale / shift: [G, D] (may be strided column chunks of one modulation tensor)."""
    if not _gpu(x):
        y = ref.layernorm_mod(x, scale, shift, rows_per_mod, eps)
        return out.copy_(y) if out is not None else y
    x2 = x if x.dim() == 2 else x.reshape(-1, x.shape[-1])
    y = out if out is not None else torch.empty(x2.shape, dtype=x.dtype, device=x.device)
    _K().layernorm_mod(x2, scale, shift, y if y.dim() == 2 else y.view(-1, x.shape[-1]), int(rows_per_mod),
                       float(eps))
    return y.view(x.shape) if out is None else out


def qk_norm_rope(x: torch.Tensor, q_w, k_w, cos, sin, heads: int, head_dim: int, seq: int, eps: float = 1e-6):
    """In place on a packed QKV buffer x [rows, >= 2*H*D]: per-head RMSNorm of q and k (weights optional) and
    pair RoPE with cos/sin [seq, D/2] (row r uses position r % seq)."""
    if not _gpu(x):
        return ref.qk_norm_rope(x, q_w, k_w, cos, sin, heads, head_dim, seq, eps)
    _K().qk_norm_rope(x, q_w, k_w, cos, sin, int(heads), int(head_dim), int(seq), float(eps))
    return x


def bmm(a: torch.Tensor, w: torch.Tensor, alpha: float = 1.0) -> torch.Tensor:
    """Batched C[b] = alpha * a[b] @ w[b]^T (a [B,M,K], w [B,N,K])."""
    if not _gpu(a):
        return (torch.matmul(a.float(), w.float().transpose(-1, -2)) * alpha).to(a.dtype)
    B, M, K = a.shape
    N = w.shape[-2]
    y = torch.empty(B, M, N, dtype=a.dtype, device=a.device)
    _K().gemm(a, w, y, None, None, 1, None, float(alpha), 1.0, ACT_NONE, False)
    return y


def set_decode_wb(mode: int = -1) -> int:
    """Decode attention routing at D 128 / GQA 4 / one split: 1 = the wave-per-block short-context kernel (default),
    0 = the split kernel (``SHAI_DECODE_WB=0``); -1 keeps the mode.  Returns the previous mode (A/B in one process)."""
    return int(_K().set_decode_wb(int(mode)))


def set_halo_conv(mode: int = -1, waves: int = -1) -> int:
    """Routing of the halo-tiled conv (csrc/kernels/conv_halo.hip): mode 0 off (default, SHAI_HALO_CONV), 1
    GroupNorm-fused convs, 2 also plain 3x3 convs; waves 4 / 8 pins its wave layout (0: default).  -1 keeps a
    setting.  Returns the previous mode (A/B in one process)."""
    return int(_K().set_halo_conv(int(mode), int(waves)))


# upsample + 3x3 conv as 4 output-phase 2x2 convs over the source (2.25x fewer MACs; SHAI_UP2_PHASES=0: off)
UP2_PHASES = os.environ.get("SHAI_UP2_PHASES", "1") != "0"
# models keep the 9-tap conv below this many 256 x 256 output tiles (``up2_phases_ok(..., cout=)``)
UP2_MIN_TILES = int(os.environ.get("SHAI_UP2_MIN_TILES", "256"))


def up2_phases_ok(x: torch.Tensor, kh: int, kw: int, stride: int, pad: int, x2=None, norm=None, residual=None,
                  cout: int = 0, temb=None) -> bool:
    """Whether an upsample conv of this shape runs phase-decomposed (v4 kernel CONV 3): plain 3x3 pad-1 conv, 64-channel
    multiples, H and W powers of two; below H W = 256 the rows run over groups of 256 / (H W) images (N a multiple,
    no per-image bias), so a 256-row tile still holds one phase.  With cout given, at least 256 output tiles: a small
    problem (SD2.1 at batch 1) stays on the 9-tap conv (measured: b32 +3.2 % img/s; b1 p50 1-1.3 % slower with every
    shape phased, split-K or not)."""
    N, H, W, C = x.shape
    if cout and (4 * N * H * W // 256) * ((cout + 255) // 256) < UP2_MIN_TILES:
        return False
    pow2 = (H & (H - 1)) == 0 and (W & (W - 1)) == 0
    grouped = H * W < 256
    return (UP2_PHASES and x.is_cuda and kh == 3 and kw == 3 and stride == 1 and pad == 1 and x2 is None and norm is None
            and residual is None and C % 64 == 0 and pow2
            and (not grouped or (N % (256 // (H * W)) == 0 and temb is None)))


def conv2d(x: torch.Tensor, w_packed: torch.Tensor, bias: Optional[torch.Tensor], kh: int, kw: int, stride: int = 1,
           pad: int = 0, upsample: bool = False, x2: Optional[torch.Tensor] = None, norm=None,
           temb: Optional[torch.Tensor] = None, residual: Optional[torch.Tensor] = None, act=None,
           res_alpha: float = 1.0, stats: Optional[str] = None, eps: float = 1e-5,
           w_up2: Optional[torch.Tensor] = None):
    """NHWC implicit-GEMM convolution with fused prologue/epilogue.

    norm = (scale [N,Cin] f32, shift [N,Cin] f32, act) applies GroupNorm(+act) to
    the input: on the GPU one vectorised apply pass + the tuned conv inside the op (``set_halo_conv(1)``: the
    halo-tiled conv normalises each staged element once in LDS instead -- measured slower at the SD2.1 shapes);
    x2 is concatenated on channels; upsample reads a
    nearest-2x view; temb [N, Cout] is a per-image bias; residual is added last.  w_up2: the phase weights
    (``pack_up2_phase_weight``) of an upsample conv -- used when ``up2_phases_ok``.
    stats="gn" / "ln": also return statistics of the output for the next norm, as ``linear_stats`` -- (out, st);
    st is None when the output shape cannot carry them (``stats_supported``).
    """
    if not _gpu(x):
        y = ref.conv2d(x, w_packed, bias, kh, kw, stride, pad, upsample, x2, norm, temb, residual, act, res_alpha)
        if stats is None:
            return y
        y2 = y.reshape(-1, y.shape[-1])
        if not stats_supported(y2.shape[0], y2.shape[1], stats, y.shape[1] * y.shape[2]):
            return y, None
        return y, (ref.row_moments(y2, eps) if stats == "ln" else ref.col_partials(y2))
    N, H, W, _ = x.shape
    IH, IW = (2 * H, 2 * W) if upsample else (H, W)
    OH = (IH + 2 * pad - kh) // stride + 1
    OW = (IW + 2 * pad - kw) // stride + 1
    cout = w_packed.shape[0]
    out = torch.empty(N, OH, OW, cout, dtype=x.dtype, device=x.device)
    sc, sh, nact = (norm if norm is not None else (None, None, None))
    M = N * OH * OW
    if stats is not None and not stats_supported(M, cout, stats, OH * OW):
        want = None
    else:
        want = stats
    gp = torch.empty(M // 128, cout, 2, dtype=torch.float32, device=x.device) if want == "gn" else None
    ls = torch.empty(M, 2, dtype=torch.float32, device=x.device) if want == "ln" else None
    if upsample and w_up2 is not None and up2_phases_ok(x, kh, kw, stride, pad, x2, norm, residual, temb=temb):
        _K().conv2d(x, None, w_up2, out, bias, temb, None, None, None, 0, 2, 2, 1, 0, True, act_id(act), 1.0, None,
                    None, gp, ls, float(eps), True)
    else:
        _K().conv2d(x, x2, w_packed, out, bias, temb, residual, sc, sh, act_id(nact), kh, kw, stride, pad,
                    bool(upsample), act_id(act), float(res_alpha), None, None, gp, ls, float(eps))
    if stats is None:
        return out
    return out, (gp if want == "gn" else ls)


# ----------------------------------------------------------------------------- attention
def attention(q, k, v, scale: Optional[float] = None, causal: bool = False, causal_offset: int = 0, kv_lens=None,
              q_lens=None, bias=None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Fused flash attention. q [B,Sq,Hq,D] (packed heads), k/v [B,Skv,Hkv,D]."""
    D = q.shape[-1]
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    if not _gpu(q):
        o = ref.attention(q, k, v, scale, causal, causal_offset, kv_lens, q_lens, bias)
        return out.copy_(o) if out is not None else o
    o = out if out is not None else torch.empty(q.shape, dtype=q.dtype, device=q.device)
    _K().flash_attn(q, k, v, o, float(scale), bool(causal), int(causal_offset), _i32(kv_lens), _i32(q_lens), bias,
                    None)
    return o


def paged_attention(q, k_cache, v_cache, block_table, kv_lens, q_lens, scale=None, causal=True):
    """Prefill attention over a paged KV cache (64-token blocks)."""
    D = q.shape[-1]
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    if not _gpu(q):
        return ref.paged_attention(q, k_cache, v_cache, block_table, kv_lens, q_lens, scale, causal)
    o = torch.empty(q.shape, dtype=q.dtype, device=q.device)
    _K().flash_attn(q, k_cache, v_cache, o, float(scale), bool(causal), 0, _i32(kv_lens), _i32(q_lens), None,
                    _i32(block_table))
    return o


def paged_attention_varlen(q, k_cache, v_cache, block_table, kv_lens, q_lens, q_start, max_q: int, scale=None,
                           causal=True):
    """Packed (varlen) prefill attention over a paged KV cache: q [T, Hq, D] holds every sequence's new tokens
    back to back (sequence b = rows q_start[b] .. + q_lens[b] - 1), so no padding rows are computed."""
    D = q.shape[-1]
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    if not _gpu(q):
        return ref.paged_attention_varlen(q, k_cache, v_cache, block_table, kv_lens, q_lens, q_start, scale, causal)
    o = torch.empty(q.shape, dtype=q.dtype, device=q.device)
    _K().paged_attn_varlen(q, k_cache, v_cache, o, _i32(block_table), _i32(kv_lens), _i32(q_lens), _i32(q_start),
                           int(max_q), float(scale), bool(causal))
    return o


# largest top-k the fused sampler keeps exactly (csrc/kernels/sampling.hip candidate buffer); rows asking for
# more (or for no top-k at all, top_k <= 0) are sampled over the full vocabulary by the torch path
SAMPLER_MAX_K = 1024


def decode_splits(batch: int, hkv: int, max_ctx: int) -> int:
    """Split-K factor of the paged decode attention: enough (sequence, KV head, split) workgroups to fill
    the chip (``SHAI_DECODE_WG`` of them, default 512 = two per CU), at most one split per 64-token block."""
    nblk = max(1, (max_ctx + 63) // 64)
    target = int(os.environ.get("SHAI_DECODE_WG", "512"))
    want = max(1, target // max(1, batch * hkv))
    return int(min(nblk, want, 64))


def decode_attention(q, k_cache, v_cache, block_table, ctx_lens, scale=None, num_splits: Optional[int] = None,
                     max_ctx: Optional[int] = None, out=None):
    """Paged single-token decode attention. q [B,Hq,D]."""
    D = q.shape[-1]
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    if not _gpu(q):
        return ref.decode_attention(q, k_cache, v_cache, block_table, ctx_lens, scale)
    B, Hq, _ = q.shape
    if num_splits is None:
        mc = max_ctx if max_ctx is not None else block_table.shape[1] * 64
        num_splits = decode_splits(B, k_cache.shape[1], mc)
    ws = torch.empty(B * Hq * num_splits * (D + 2), dtype=torch.float32, device=q.device)
    o = out if out is not None else torch.empty(q.shape, dtype=q.dtype, device=q.device)
    _K().decode_attn(q, k_cache, v_cache, o, _i32(block_table), _i32(ctx_lens), ws, int(num_splits), float(scale))
    return o


def decode_attention_rope(qkv, k_cache, v_cache, block_table, ctx_lens, positions, cos, sin, slots, h: int, hk: int,
                          scale=None, num_splits: Optional[int] = None, max_ctx: Optional[int] = None, out=None):
    """One fused decode step on the packed QKV rows qkv [B, (h + 2 hk) D]: NeoX RoPE on q / k, this step's k / v
    written into the paged caches at ``slots`` (-1: padding row), attention over the cached context plus the
    new token (``ctx_lens`` count it).  Equivalent to rope_qkv_cache + decode_attention.  Returns [B, h D]."""
    D = k_cache.shape[-1]
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    B = qkv.shape[0]
    if not _gpu(qkv):
        rope_qkv_cache(qkv, positions, cos, sin, k_cache, v_cache, slots, h, hk)
        q = qkv[:, : h * D].reshape(B, h, D)
        return decode_attention(q, k_cache, v_cache, block_table, ctx_lens, scale).reshape(B, h * D)
    if num_splits is None:
        mc = max_ctx if max_ctx is not None else block_table.shape[1] * 64
        num_splits = decode_splits(B, hk, mc)
    ws = torch.empty(B * h * num_splits * (D + 2), dtype=torch.float32, device=qkv.device)
    o = out if out is not None else torch.empty(B, h * D, dtype=qkv.dtype, device=qkv.device)
    _K().decode_attn_rope(qkv, k_cache, v_cache, o, _i32(block_table), _i32(ctx_lens), _i32(positions), cos, sin,
                          _i32(slots), ws, int(h), int(hk), int(num_splits), float(scale))
    return o


def gemm_partials(x, w, rms_eps: float) -> torch.Tensor:
    """Decode-shaped x [M <= 64, K] times w [N, K]^T with the folded RMSNorm of x, left UNFOLDED: the skinny
    kernel's split-K fp32 partials [kg][M][N] followed by the [kg][M] row sums of squares (kg = numel / (M (N + 1)),
    at least 2).  decode_attention_rope_qkv folds them (no separate reduce launch)."""
    return _K().gemm_partials(x, w, float(rms_eps))


def decode_attention_rope_qkv(x, w_qkv, rms_eps: float, k_cache, v_cache, block_table, ctx_lens, positions, cos, sin,
                              slots, h: int, hk: int, scale=None, num_splits: Optional[int] = None, out=None):
    """decode_attention_rope on qkv = linear(rmsnorm(x), w_qkv) (norm gain folded into w_qkv) with the QKV GEMM's
    split-K fold done inside the attention kernel.  Same values as the two-step form: the kernel adds the partial
    slabs in the fold's order and rounds q / k / v to bf16 as the fold's epilogue does.  Returns [B, h D]."""
    if not _gpu(x):
        return decode_attention_rope(linear(x, w_qkv, rms_eps=rms_eps), k_cache, v_cache, block_table, ctx_lens,
                                     positions, cos, sin, slots, h, hk, scale, num_splits, out=out)
    D = k_cache.shape[-1]
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    B, K = x.shape
    N = w_qkv.shape[0]
    if num_splits is None:
        num_splits = decode_splits(B, hk, block_table.shape[1] * 64)
    part = gemm_partials(x, w_qkv, rms_eps)
    kg = part.numel() // (B * (N + 1))
    ws = torch.empty(B * h * num_splits * (D + 2), dtype=torch.float32, device=x.device)
    o = out if out is not None else torch.empty(B, h * D, dtype=x.dtype, device=x.device)
    # qkv slot: the (read-only) partials stand in -- never an alias of the mutated output o
    _K().decode_attn_rope(part, k_cache, v_cache, o, _i32(block_table), _i32(ctx_lens), _i32(positions), cos, sin,
                          _i32(slots), ws, int(h), int(hk), int(num_splits), float(scale), part, int(kg), int(K),
                          float(rms_eps))
    return o


def kv_write(k, v, k_cache, v_cache, slots):
    if not _gpu(k):
        return ref.kv_write(k, v, k_cache, v_cache, slots)
    _K().kv_write(k, v, k_cache, v_cache, _i32(slots))


# ----------------------------------------------------------------------------- elementwise
def rope(x, positions, cos, sin, rot_dim: Optional[int] = None, neox: bool = True):
    """In-place rotary embedding on x [T, H, Dh] (token stride may be > H*Dh)."""
    rot = rot_dim if rot_dim is not None else x.shape[-1]
    if not _gpu(x):
        return ref.rope(x, positions, cos, sin, rot, neox)
    _K().rope(x, _i32(positions), cos, sin, int(rot), bool(neox))
    return x


def rope_qkv_cache(qkv, positions, cos, sin, k_cache, v_cache, slots, heads: int, kv_heads: int):
    """Packed QKV rows [T, (H + 2Hkv) * D]: NeoX RoPE on q in place, rotated k and v written to the paged
    caches [blocks, Hkv, 64, D] at ``slots`` (-1 = skip).  One fused kernel on the GPU."""
    T = qkv.shape[0]
    D = k_cache.shape[-1]
    if not _gpu(qkv):
        q = qkv[:, : heads * D].view(T, heads, D)
        k = qkv[:, heads * D:(heads + kv_heads) * D].view(T, kv_heads, D)
        v = qkv[:, (heads + kv_heads) * D:].view(T, kv_heads, D)
        ref.rope(q, positions, cos, sin, D, True)
        ref.rope(k, positions, cos, sin, D, True)
        ref.kv_write(k, v, k_cache, v_cache, slots)
        return qkv
    _K().rope_qkv_cache(qkv, _i32(positions), cos, sin, k_cache, v_cache, _i32(slots), int(heads), int(kv_heads))
    return qkv


def sample(logits, temps, top_k, top_p, uniforms, out):
    """Fused temperature / top-k / top-p sampling (GPU only; one workgroup per row)."""
    _K().sample(logits, temps, top_k, top_p, uniforms, out)
    return out


def rope_pairs(x, cos, sin):
    """In-place Flux RoPE on x [B, T, H, Dh] with cos/sin [T, Dh/2]."""
    if not _gpu(x):
        return ref.rope_pairs(x, cos, sin)
    _K().rope_pairs(x, cos, sin)
    return x


def gated_act(x, act="silu", gate_first: bool = False):
    """[.., 2F] -> [.., F]: a*act(g) (gate_first: act(a)*g)."""
    if not _gpu(x):
        return ref.gated_act(x, act, gate_first)
    F_ = x.shape[-1] // 2
    out = torch.empty(*x.shape[:-1], F_, dtype=x.dtype, device=x.device)
    x2 = x if x.dim() == 2 else x.reshape(-1, x.shape[-1])
    _K().gated_act(x2, out.view(-1, F_), act_id(act), bool(gate_first))
    return out


def bias_act(x, bias=None, residual=None, act=None, alpha: float = 1.0):
    if not _gpu(x):
        return ref.bias_act(x, bias, residual, act, alpha)
    x = x.contiguous()
    out = torch.empty_like(x)
    _K().bias_act(x, bias, residual.contiguous() if residual is not None else None, out, act_id(act), float(alpha))
    return out


def sched_step(model_out, latents, cfg: bool, guidance: float, pred_type: int, a_t: float, a_prev: float,
               dt: float = 0.0):
    """Fused CFG + scheduler update, in place on latents."""
    if not _gpu(latents):
        return ref.sched_step(model_out, latents, cfg, guidance, pred_type, a_t, a_prev, dt)
    _K().sched_step(model_out, latents, bool(cfg), float(guidance), int(pred_type), float(a_t), float(a_prev),
                    float(dt))
    return latents


def sched_step_rows(model_out, latents, cfg: bool, guidance: float, pred_type: int, rows_params):
    """Per-row fused CFG + scheduler update (step-level batching): latents [B, ...], every row at its own step;
    rows_params fp32 [B, 3] = (a_t, a_prev, dt) per row, a_t < 0 marks an idle row (left unchanged)."""
    if not _gpu(latents):
        return ref.sched_step_rows(model_out, latents, cfg, guidance, pred_type, rows_params)
    _K().sched_step_rows(model_out, latents, bool(cfg), float(guidance), int(pred_type), rows_params.contiguous())
    return latents


def softmax_(x, scale: float = 1.0):
    if not _gpu(x):
        x.copy_(torch.softmax(x.float() * scale, dim=-1).to(x.dtype))
        return x
    _K().softmax_(x, float(scale))
    return x


def token_feedback(ids, rowmap, prev):
    """In place: ids[i] = prev[rowmap[i]] where rowmap[i] >= 0 (decode-step token feedback; all int32)."""
    if not _gpu(ids):
        prev_rows = prev.index_select(0, rowmap.clamp(min=0).long())
        ids.copy_(torch.where(rowmap >= 0, prev_rows, ids))
        return ids
    _K().token_feedback(ids, rowmap, prev)
    return ids


def embedding(ids, table):
    if not _gpu(table):
        return table[ids.long()]
    out = torch.empty(*ids.shape, table.shape[1], dtype=table.dtype, device=table.device)
    _K().embedding(_i32(ids).contiguous(), table, out)
    return out
