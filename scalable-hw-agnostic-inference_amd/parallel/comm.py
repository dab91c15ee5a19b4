"""Tensor-parallel collectives.

Issued on the current stream, so they are ordered with the surrounding kernels
and capturable in HIP graphs.  Two transports:

* RCCL (``torch.distributed`` backend "nccl" on ROCm) -- default for every size;
  also the sequence-parallel all-gather / reduce-scatter pair (:func:`all_gather_seq`,
  :func:`reduce_scatter_seq`) used by the Flux single-stream blocks at SP > 1.
* ``P2PAllReduce`` (``csrc/comm/p2p_allreduce.hip``) -- xGMI peer-memory kernels
  over IPC-mapped buffers, ON by default for every TP > 1 group on GPUs
  (``SHAI_P2P_ALLREDUCE=0`` disables it).  Routing by message size:
  one-shot (every rank reads every peer's whole message; latency-bound LLM decode,
  B x 4096 bf16) up to ``SHAI_P2P_ONE_SHOT_MAX`` (256 KiB), two-shot
  (reduce-scatter + all-gather over all 7 links at once; Flux / prefill
  row-parallel outputs, 27 MiB per call for Flux 1024^2 at TP8) up to
  ``SHAI_P2P_MAX_BYTES`` (32 MiB, the staging capacity), RCCL above; a one-shot all-gather for vocab-parallel logits.
  A row-parallel layer (:func:`row_parallel_reduce`) writes its GEMM partial
  straight into this rank's IPC staging slot and one fused kernel reduces it and
  adds the bias and the residual (no staging copy, no separate residual launch);
  large outputs are split into row slabs whose reduces overlap the next slab's GEMM.
  A peer that never arrives sets an error word the engines poll after every step
  (:func:`raise_if_p2p_error`).

On a fully connected 8x MI355X node each GPU has 7 xGMI links; RCCL's
multi-channel rings / direct algorithms use them for the large Flux/prefill
messages, the one-shot kernel removes the ring latency for the small ones.
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.distributed as dist

from .state import tp

_P2P = None
P2P_ONE_SHOT_MAX = int(os.environ.get("SHAI_P2P_ONE_SHOT_MAX", str(256 * 1024)))
P2P_CAPACITY = int(os.environ.get("SHAI_P2P_CAPACITY", str(32 << 20)))   # Flux 1024^2 TP8 messages: 27 MiB
P2P_MAX_BYTES = int(os.environ.get("SHAI_P2P_MAX_BYTES", str(P2P_CAPACITY)))
# SHAI_P2P_STAGED=0: row-parallel layers all-reduce a separate GEMM output (staging copy + residual launch)
P2P_STAGED = os.environ.get("SHAI_P2P_STAGED", "1") != "0"


def enable_p2p(p2p) -> None:
    global _P2P
    _P2P = p2p


def p2p():
    return _P2P


def raise_if_p2p_error() -> None:
    """Raise if an xGMI peer collective timed out (a peer never arrived): its output is a partial sum.
    Reads a host-mapped word -- no device synchronisation -- so the engines call it after every step."""
    if _P2P is not None and _P2P.error():
        # the error word is never cleared (the peer buffers may hold a half-finished round): the process is
        # done serving -- /health turns 503 for good and the supervisor restarts the TP group
        from ..utils.liveness import mark_broken
        msg = "xGMI P2P collective timed out waiting for a peer rank: TP group broken"
        mark_broken(msg)
        raise RuntimeError(msg)


def all_reduce(x: torch.Tensor, group: Optional[dist.ProcessGroup] = None) -> torch.Tensor:
    """In-place sum over the TP group (no-op at TP=1)."""
    st = tp()
    g = group if group is not None else st.group
    if st.size == 1 and group is None:
        return x
    if _P2P is not None and x.is_cuda and x.numel() * x.element_size() <= _P2P.max_bytes and x.is_contiguous():
        return _P2P.all_reduce(x)
    dist.all_reduce(x, group=g)
    return x


# Row-parallel output stage: fused AND overlapped.  A RowParallel GEMM with at least
# OVERLAP_MIN_ROWS rows is split into OVERLAP_CHUNKS row slabs; slab i's GEMM writes its partial product into its own
# region of this rank's IPC staging slot, and slab i's staged reduce (one-shot or two-shot by slab size, with the
# bias / AdaLN gate / residual epilogue fused) runs on a side stream while slab i + 1's GEMM runs on the compute
# stream.  Fork / join by events, so it is HIP-graph capturable; every slab is its own collective, issued in the
# same order on every rank.
_env_chunks = os.environ.get("SHAI_TP_OVERLAP_CHUNKS")
OVERLAP_CHUNKS: Optional[int] = int(_env_chunks) if _env_chunks else None   # None: by rows and message size
OVERLAP_MIN_ROWS = int(os.environ.get("SHAI_TP_OVERLAP_MIN_ROWS", "1024"))
OVERLAP_MIN_BYTES = int(os.environ.get("SHAI_TP_OVERLAP_MIN_BYTES", str(2 << 20)))
_SIDE: dict = {}


def _side_stream(device: torch.device) -> "torch.cuda.Stream":
    idx = device.index if device.index is not None else torch.cuda.current_device()
    if idx not in _SIDE:
        _SIDE[idx] = torch.cuda.Stream(device=idx)
    return _SIDE[idx]


def overlap_chunks(rows: int, cols: int = 0, elem_bytes: int = 2) -> int:
    """How many row slabs a row-parallel GEMM of ``rows`` x ``cols`` outputs is split into (1: no overlap).

    Only the LAST slab's reduce is exposed after the GEMM, so the exposed share of the message is 1 / slabs, while
    every slab GEMM must still fill the chip: 4 slabs from 4096 rows (Flux 1024^2: 4608 rows, 27 MiB per call at
    TP8 -> ~6.8 MiB exposed instead of 13.5 with 2), 2 from OVERLAP_MIN_ROWS (1024: Flux 512^2, LLM prefill
    chunks), none below it or for messages under OVERLAP_MIN_BYTES (latency-bound reduces: a split only adds
    launches).  SHAI_TP_OVERLAP_CHUNKS (or setting ``OVERLAP_CHUNKS``) pins the count for every large message."""
    if tp().size == 1 or rows < OVERLAP_MIN_ROWS:
        return 1
    if OVERLAP_CHUNKS is not None:
        return max(1, min(OVERLAP_CHUNKS, rows))
    if cols and rows * cols * elem_bytes < OVERLAP_MIN_BYTES:
        return 1
    return 4 if rows >= 4096 else 2


def row_slabs(rows: int, chunks: int):
    """[(r0, r1), ...]: the row slabs of a ``chunks``-way split (equal slabs, the last one ragged)."""
    chunks = max(1, min(chunks, rows))
    step = (rows + chunks - 1) // chunks
    return [(r, min(rows, r + step)) for r in range(0, rows, step)]


def _epilogue_rows(y: torch.Tensor, out: torch.Tensor, bias, residual, gate, rows_per_gate: int, row0: int) -> None:
    """out = residual + gate[(row0 + r) // rows_per_gate] * (y + bias) for a slab of rows (host reference of the
    fused staged-reduce epilogue, p2p_allreduce.hip apply_epi)."""
    v = y.float()
    if bias is not None:
        v = v + bias.float()
    if gate is not None:
        idx = torch.div(torch.arange(row0, row0 + y.shape[0], device=y.device), rows_per_gate, rounding_mode="floor")
        v = v * gate[idx, : y.shape[1]].float()
    if residual is not None:
        v = v + residual.float()
    out.copy_(v.to(out.dtype))


def _al16(t: Optional[torch.Tensor]) -> bool:
    return t is None or t.data_ptr() % 16 == 0


def _staged_ok(p, x, rows, n, w_scale, residual, out, bias, gate2) -> bool:
    """Whether the fused staged P2P reduce (GEMM into the IPC slot + one reduce/epilogue kernel) takes a message."""
    if p is None or not P2P_STAGED or x.dtype != torch.bfloat16:
        return False
    if n % 8 or rows * n * 2 > p.max_bytes or (w_scale is not None and rows > 64):
        return False
    for t in (residual, out, bias):
        if t is not None and (t.dtype != torch.bfloat16 or not _al16(t)):
            return False
    if bias is not None and (not bias.is_contiguous() or bias.numel() != n):
        return False
    if gate2 is not None and (gate2.dtype != torch.bfloat16 or gate2.stride(-1) != 1 or gate2.shape[-1] < n
                              or gate2.stride(0) % 8 or not _al16(gate2)):
        return False
    return True


def _generic_slabs(x, x2, weight, bias, residual, w_scale, gate2, rows_per_gate, out, bounds):
    """Overlapped row-parallel stage without the staged P2P reduce (no P2P group, a message above its capacity,
    fp8 prefill): slab i's GEMM runs on the compute stream while slab i - 1's all-reduce (RCCL, or the unstaged P2P
    kernels) and its bias / gate / residual epilogue run on the side stream."""
    from .. import ops
    n = weight.shape[0]
    rows = x2.shape[0]
    if out is None:
        out = torch.empty(*x.shape[:-1], n, dtype=x.dtype, device=x.device)
    o2 = out.view(rows, n)
    r2 = residual.reshape(rows, n) if residual is not None else None
    cur = torch.cuda.current_stream(x.device)
    side = _side_stream(x.device)
    side.wait_stream(cur)
    for r0, r1 in bounds:
        ys = ops.linear(x2[r0:r1], weight, None, w_scale=w_scale)
        ev = torch.cuda.Event()
        ev.record(cur)
        side.wait_event(ev)
        ys.record_stream(side)   # allocated on the compute stream, consumed on the side stream
        with torch.cuda.stream(side):
            all_reduce(ys)
            _epilogue_rows(ys, o2[r0:r1], bias, r2[r0:r1] if r2 is not None else None, gate2, rows_per_gate, r0)
    cur.wait_stream(side)
    return out


def row_parallel_reduce(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor],
                        residual: Optional[torch.Tensor], w_scale: Optional[torch.Tensor] = None,
                        gate: Optional[torch.Tensor] = None, rows_per_gate: int = 1,
                        out: Optional[torch.Tensor] = None, chunks: int = 1) -> Optional[torch.Tensor]:
    """Fused output stage of a row-parallel layer: out = residual + gate[row // rows_per_gate] * (sum over the TP
    group of x @ weight^T + bias), ``out`` may be ``residual`` (the in-place gated update of the Flux blocks).

    xGMI P2P (GPU): the GEMM writes this rank's partial product ([..., N], x's leading shape) straight into the IPC
    staging slot and ONE kernel per slab sums every rank's slot region (one-shot or two-shot by size) and applies
    the epilogue; with ``chunks`` > 1 the slabs' reduces overlap the next slabs' GEMMs (side stream).  CPU (gloo):
    the same slab schedule with an all-reduce per slab and the epilogue in torch.  Returns None when the message
    does not qualify (no P2P, too large, fp8 prefill, odd widths, strided or unaligned tensors); the caller then
    takes the generic GEMM -> all_reduce -> epilogue path."""
    n = weight.shape[0]
    rows = x.numel() // x.shape[-1]
    x2 = x.reshape(rows, x.shape[-1])
    for t in (residual, out):
        if t is not None and (t.numel() != rows * n or not t.is_contiguous()):
            return None
    gate2 = gate.reshape(-1, gate.shape[-1]) if gate is not None else None
    bounds = row_slabs(rows, chunks)
    if not x.is_cuda:
        from .. import ops
        if out is None:
            out = torch.empty(*x.shape[:-1], n, dtype=x.dtype, device=x.device)
        o2, r2 = out.view(rows, n), residual.reshape(rows, n) if residual is not None else None
        for r0, r1 in bounds:
            y = ops.linear(x2[r0:r1], weight, None, w_scale=w_scale)
            all_reduce(y)
            _epilogue_rows(y, o2[r0:r1], bias, r2[r0:r1] if r2 is not None else None, gate2, rows_per_gate, r0)
        return out
    p = _P2P
    if not _staged_ok(p, x, rows, n, w_scale, residual, out, bias, gate2):
        # no staged P2P reduce for this message: with several slabs, the generic overlapped slab loop (GEMM per
        # slab on the compute stream, that slab's all-reduce + epilogue on the side stream); one slab -> the
        # caller's serial GEMM -> all_reduce -> epilogue path
        if len(bounds) == 1:
            return None
        return _generic_slabs(x, x2, weight, bias, residual, w_scale, gate2, rows_per_gate, out, bounds)
    from .. import ops
    stage = p.staging(rows, n, x.device)
    if out is None:
        out = torch.empty(*x.shape[:-1], n, dtype=x.dtype, device=x.device)
    o2 = out.view(rows, n)
    r2 = residual.view(rows, n) if residual is not None else None
    if len(bounds) == 1:
        ops.gemm_into(x2, weight, stage, w_scale=w_scale)
        p.reduce_staged(o2, n, bias, r2, gate2, rows_per_gate)
        return out
    cur = torch.cuda.current_stream(x.device)
    side = _side_stream(x.device)
    side.wait_stream(cur)   # out / residual / gate are ready before the side stream touches them
    for r0, r1 in bounds:
        ops.gemm_into(x2[r0:r1], weight, stage[r0:r1], w_scale=w_scale)
        ev = torch.cuda.Event()
        ev.record(cur)
        side.wait_event(ev)
        with torch.cuda.stream(side):
            p.reduce_staged(o2[r0:r1], n, bias, r2[r0:r1] if r2 is not None else None, gate2, rows_per_gate,
                            row0=r0, slot_off=r0 * n * 2)
    cur.wait_stream(side)
    return out


def all_gather_last(x: torch.Tensor, group: Optional[dist.ProcessGroup] = None) -> torch.Tensor:
    """Concatenate the TP shards along the last dim."""
    st = tp()
    g = group if group is not None else st.group
    if st.size == 1 and group is None:
        return x
    n = st.size if group is None else dist.get_world_size(g)
    x = x.contiguous()
    flat = torch.empty((n * x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    if (group is None and _P2P is not None and x.is_cuda and x.dtype == torch.bfloat16
            and _P2P.can_gather(x.numel() * x.element_size())):
        _P2P.all_gather_into(flat, x)                  # one-shot over xGMI (vocab-parallel logits)
    else:
        dist.all_gather_into_tensor(flat, x, group=g)   # rank-major concat along dim 0
    out = flat.view((n,) + tuple(x.shape))
    return out.movedim(0, -2).reshape(*x.shape[:-1], n * x.shape[-1])


def _seq_major(x: torch.Tensor, n: int) -> torch.Tensor:
    """[B, n*s, ...] -> rank-major contiguous [n, B, s, ...] (a view when B == 1)."""
    B, S = x.shape[0], x.shape[1]
    return x.reshape(B, n, S // n, *x.shape[2:]).transpose(0, 1).contiguous()   # no copy when B == 1


def all_gather_seq(x: torch.Tensor, group: Optional[dist.ProcessGroup] = None) -> torch.Tensor:
    """Sequence-parallel all-gather: local [B, s, ...] shards -> [B, n*s, ...] (rank r owns rows
    [r*s, (r+1)*s)).  One all-gather of B*S*d elements; at B == 1 the rank-major result IS the output layout,
    so no re-layout copy is made."""
    st = tp()
    g = group if group is not None else st.group
    if st.size == 1 and group is None:
        return x
    n = st.size if group is None else dist.get_world_size(g)
    x = x.contiguous()
    B, s = x.shape[0], x.shape[1]
    flat = torch.empty((n * B,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    dist.all_gather_into_tensor(flat, x, group=g)   # rank-major along dim 0
    if B == 1:
        return flat.view((1, n * s) + tuple(x.shape[2:]))
    return flat.view((n,) + tuple(x.shape)).transpose(0, 1).reshape((B, n * s) + tuple(x.shape[2:]))


SP_GATHER_OVERLAP = os.environ.get("SHAI_SP_GATHER_OVERLAP", "1") != "0"


def gather_seq_linears(x: torch.Tensor, specs, group: Optional[dist.ProcessGroup] = None) -> None:
    """Sequence-parallel all-gather fused with the column-parallel GEMMs that consume it (fork / join):
    ``out = act(gather_seq(x) @ w^T + b)`` for every ``(w, b, act, out)`` in ``specs``, ``out`` a [B, n*s, N] view.

    The all-gather is issued asynchronously (RCCL runs it on its own stream; gloo on its worker thread) and this
    rank's own s rows -- already local -- go through every GEMM while the other ranks' rows are in flight; after
    the join, the rows of the ranks before and after this one run as one batched GEMM each per image ([r, s, d]
    views of the rank-major gather buffer, no re-layout copy).  On xGMI's full mesh the gather is one direct
    exchange with every peer, so the own-rows GEMMs are what it can hide behind.  Reference: the Flux single
    blocks' column-parallel QKV / MLP after the sequence gather (app/src/transformer/model.py:303-322);
    SHAI_SP_GATHER_OVERLAP=0 gathers first (A/B)."""
    from .. import ops
    st = tp()
    g = group if group is not None else st.group
    n = st.size if group is None else (dist.get_world_size(g) if dist.is_initialized() else 1)
    if n == 1 or not SP_GATHER_OVERLAP:
        xg = all_gather_seq(x, group) if n > 1 else x
        for w, b, act, out in specs:
            ops.gemm_into(xg, w, out, b, act=act)
        return
    r = dist.get_rank(g)
    x = x.contiguous()
    B, s = x.shape[0], x.shape[1]
    flat = torch.empty((n * B,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    work = dist.all_gather_into_tensor(flat, x, group=g, async_op=True)   # rank-major along dim 0
    for w, b, act, out in specs:                                           # own rows beside the exchange
        ops.gemm_into(x, w, out[:, r * s:(r + 1) * s], b, act=act)
    work.wait()
    fv = flat.view((n, B) + tuple(x.shape[1:]))
    for w, b, act, out in specs:
        N = out.shape[-1]
        for bi in range(B):
            for j0, j1 in ((0, r), (r + 1, n)):
                if j1 > j0:
                    ops.gemm_into(fv[j0:j1, bi], w, out[bi, j0 * s:j1 * s].view(j1 - j0, s, N), b, act=act)


def reduce_scatter_seq(x: torch.Tensor, group: Optional[dist.ProcessGroup] = None) -> torch.Tensor:
    """Sequence-parallel reduce-scatter: partial sums [B, S, ...] -> this rank's reduced rows [B, S/n, ...].
    Replaces the all-reduce after a RowParallel layer (same bytes on the wire as the all-gather that feeds
    the next ColumnParallel layer; together they cost one all-reduce, but every norm / residual between
    them touches only S/n rows).  gloo has no reduce-scatter: there it is all-reduce + slice."""
    st = tp()
    g = group if group is not None else st.group
    if st.size == 1 and group is None:
        return x
    n = st.size if group is None else dist.get_world_size(g)
    r = dist.get_rank(g)
    B, S = x.shape[0], x.shape[1]
    assert S % n == 0, f"sequence {S} not divisible by the SP degree {n}"
    s = S // n
    if dist.get_backend(g) == "gloo":
        y = x.clone(memory_format=torch.contiguous_format)   # never reduce into the caller's partial sums
        dist.all_reduce(y, group=g)
        return y[:, r * s:(r + 1) * s].contiguous()
    src = _seq_major(x, n)
    out = torch.empty((B, s) + tuple(x.shape[2:]), dtype=x.dtype, device=x.device)
    dist.reduce_scatter_tensor(out, src, group=g)
    return out


def broadcast_object(obj, src: int = 0):
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return obj
    lst = [obj]
    dist.broadcast_object_list(lst, src=src)
    return lst[0]


class P2PAllReduce:
    """bf16 all-reduce over IPC-mapped peer buffers (csrc/comm/p2p_allreduce.hip): one-shot (every rank
    reads every peer's whole message) up to ``one_shot_max`` bytes, two-shot (reduce-scatter + all-gather
    over all xGMI links at once) up to ``max_bytes``.

    Built once per TP group (handles exchanged with ``all_gather_object``), then used by
    :func:`all_reduce` for contiguous bf16 messages once registered with :func:`enable_p2p`
    (``SHAI_P2P_ALLREDUCE=1`` in the engine).  Everything larger, or any other dtype, goes to RCCL."""

    def __init__(self, group: Optional[dist.ProcessGroup] = None, max_bytes: int = P2P_MAX_BYTES,
                 one_shot_max: int = P2P_ONE_SHOT_MAX, capacity: Optional[int] = None):
        import ctypes
        from .. import native
        self.lib = native.comm()
        self.lib.shai_p2p_create.restype = ctypes.c_void_p
        self.lib.shai_p2p_create.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_char_p]
        self.lib.shai_p2p_open.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
        for fn in (self.lib.shai_p2p_allreduce_bf16, self.lib.shai_p2p_allreduce2_bf16, self.lib.shai_p2p_allgather):
            fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
        self.one_shot_max = one_shot_max
        self.lib.shai_p2p_staging.restype = ctypes.c_void_p
        self.lib.shai_p2p_staging.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_size_t)]
        self.lib.shai_p2p_allreduce_staged.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                                       ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                                       ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        self.lib.shai_p2p_allreduce_staged_at.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                                          ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                                          ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                          ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
        self.lib.shai_p2p_launch_counts.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_longlong)]
        self.lib.shai_p2p_error.argtypes = [ctypes.c_void_p]
        self.lib.shai_p2p_set_max_blocks.argtypes = [ctypes.c_void_p, ctypes.c_int]
        self.lib.shai_p2p_destroy.argtypes = [ctypes.c_void_p]
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.max_bytes = max_bytes                       # all-reduce routing threshold
        self.capacity = max(max_bytes, capacity if capacity is not None else P2P_CAPACITY)   # staging slot size
        hs = self.lib.shai_p2p_handle_size()
        buf = ctypes.create_string_buffer(hs)
        self.ctx = self.lib.shai_p2p_create(self.rank, self.world, self.capacity, buf)
        if not self.ctx:
            raise RuntimeError("P2P all-reduce buffer allocation / IPC export failed")
        handles = [None] * self.world
        dist.all_gather_object(handles, bytes(buf.raw), group=group)
        rc = self.lib.shai_p2p_open(self.ctx, b"".join(handles))
        if rc != 0:
            raise RuntimeError(f"hipIpcOpenMemHandle failed for peer {-rc - 1}")
        # ranks sharing one GPU (tests) must all be resident at once: SHAI_P2P_MAX_BLOCKS caps every grid
        if os.environ.get("SHAI_P2P_MAX_BLOCKS"):
            self.lib.shai_p2p_set_max_blocks(self.ctx, int(os.environ["SHAI_P2P_MAX_BLOCKS"]))
        dist.barrier(group=group)

    def all_reduce(self, x: torch.Tensor) -> torch.Tensor:
        nbytes = x.numel() * x.element_size()
        if x.dtype != torch.bfloat16 or not x.is_contiguous() or nbytes % 16 or nbytes > self.max_bytes:
            dist.all_reduce(x, group=self.group)
            return x
        st = torch.cuda.current_stream(x.device).cuda_stream
        fn = self.lib.shai_p2p_allreduce_bf16 if nbytes <= self.one_shot_max else self.lib.shai_p2p_allreduce2_bf16
        rc = fn(self.ctx, x.data_ptr(), x.data_ptr(), nbytes, st)
        if rc != 0:
            raise RuntimeError(f"p2p all-reduce launch failed ({rc})")
        return x

    def staging(self, rows: int, cols: int, device) -> torch.Tensor:
        """A bf16 [rows, cols] view of this rank's IPC staging slot (the GEMM output of :meth:`reduce_staged`).
        One slot per group: valid until the next collective of this group."""
        import ctypes
        cap = ctypes.c_size_t(0)
        ptr = self.lib.shai_p2p_staging(self.ctx, ctypes.byref(cap))
        assert rows * cols * 2 <= cap.value
        idx = device.index if getattr(device, "index", None) is not None else torch.cuda.current_device()
        from .. import native
        return native.ops().from_ptr(int(ptr), [rows, cols], torch.bfloat16, int(idx))

    def reduce_staged(self, out: torch.Tensor, ncols: int, bias: Optional[torch.Tensor] = None,
                      residual: Optional[torch.Tensor] = None, gate: Optional[torch.Tensor] = None,
                      rows_per_gate: int = 1, row0: int = 0, slot_off: int = 0) -> torch.Tensor:
        """out = residual + gate[(row0 + row) // rows_per_gate] * (sum over ranks of the staged partials + bias)
        (contiguous bf16, ``out.numel()`` elements at byte ``slot_off`` of every rank's staging slot -- a row slab
        of a larger staged output; ``out`` may be ``residual``; ``gate`` [G, >= ncols] with rows of stride
        ``gate.stride(0)``)."""
        nbytes = out.numel() * 2
        two = nbytes > self.one_shot_max
        for t in (bias, residual):
            assert t is None or (t.dtype == torch.bfloat16 and t.is_contiguous())
        if gate is not None:
            assert gate.dtype == torch.bfloat16 and gate.dim() == 2 and gate.stride(1) == 1
        st = torch.cuda.current_stream(out.device).cuda_stream
        rc = self.lib.shai_p2p_allreduce_staged_at(self.ctx, out.data_ptr(), nbytes, int(ncols),
                                                   bias.data_ptr() if bias is not None else None,
                                                   residual.data_ptr() if residual is not None else None,
                                                   gate.data_ptr() if gate is not None else None,
                                                   int(gate.stride(0)) if gate is not None else 0, int(rows_per_gate),
                                                   int(row0), int(slot_off), int(two), st)
        if rc != 0:
            raise RuntimeError(f"p2p staged all-reduce launch failed ({rc})")
        return out

    def launch_counts(self) -> dict:
        """Kernel launches per algorithm so far (a captured launch counts once)."""
        import ctypes
        buf = (ctypes.c_longlong * 5)()
        self.lib.shai_p2p_launch_counts(self.ctx, buf)
        return dict(zip(("one_shot", "two_shot", "staged_one_shot", "staged_two_shot", "all_gather"), list(buf)))

    def can_gather(self, shard_bytes: int) -> bool:
        return shard_bytes % 16 == 0 and shard_bytes <= self.capacity

    def all_gather_into(self, out: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
        """Rank-major concatenation of every rank's contiguous bf16 ``x`` into ``out`` ([world * rows, ...])."""
        st = torch.cuda.current_stream(x.device).cuda_stream
        rc = self.lib.shai_p2p_allgather(self.ctx, x.data_ptr(), out.data_ptr(), x.numel() * x.element_size(), st)
        if rc != 0:
            raise RuntimeError(f"p2p all-gather launch failed ({rc})")
        return out

    def error(self) -> bool:
        return bool(self.lib.shai_p2p_error(self.ctx))

    def close(self):
        if self.ctx:
            self.lib.shai_p2p_destroy(self.ctx)
            self.ctx = None
