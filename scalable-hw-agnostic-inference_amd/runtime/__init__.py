"""ctypes bindings of the native host runtime (``csrc/runtime``): paged-KV block
manager with prefix caching and the continuous-batching scheduler helpers."""
from __future__ import annotations

import ctypes
from typing import List, Sequence

import numpy as np

from .. import native

_I = ctypes.c_int
_P = ctypes.c_void_p
_IP = ctypes.POINTER(ctypes.c_int)
_U64P = ctypes.POINTER(ctypes.c_uint64)
_I64P = ctypes.POINTER(ctypes.c_int64)
_lib = None


def lib():
    global _lib
    if _lib is None:
        L = native.runtime()
        L.shai_bm_create.restype = _P
        L.shai_bm_create.argtypes = [_I]
        L.shai_bm_destroy.argtypes = [_P]
        L.shai_bm_num_free.argtypes = [_P]
        L.shai_bm_num_free.restype = _I
        L.shai_bm_num_blocks.argtypes = [_P]
        L.shai_bm_allocate.argtypes = [_P, _I, _IP]
        L.shai_bm_allocate.restype = _I
        L.shai_bm_fork.argtypes = [_P, _IP, _I]
        L.shai_bm_release.argtypes = [_P, _IP, _I]
        L.shai_bm_register.argtypes = [_P, _I, ctypes.c_uint64]
        L.shai_bm_lookup_prefix.argtypes = [_P, _U64P, _I, _IP]
        L.shai_bm_lookup_prefix.restype = _I
        L.shai_bm_stats.argtypes = [_P, _I64P]
        L.shai_bm_refcount.argtypes = [_P, _I]
        L.shai_bm_refcount.restype = _I
        L.shai_sched_admit.argtypes = [_I, _IP, _I, _I, _I, _I, _I]
        L.shai_sched_admit.restype = _I
        L.shai_build_decode.argtypes = [_I, _IP, _IP, _IP, _I, _IP, _IP, _IP, _IP]
        L.shai_build_prefill.argtypes = [_I, _I, _IP, _IP, _IP, _IP, _I, _IP, _IP, _IP, _IP, _IP, _IP]
        L.shai_build_prefill_packed.argtypes = [_I, _IP, _IP, _IP, _IP, _I, _IP, _IP, _IP, _IP, _IP, _IP, _IP]
        _lib = L
    return _lib


def _ip(a: np.ndarray):
    assert a.dtype == np.int32 and a.flags.c_contiguous
    return a.ctypes.data_as(_IP)


class BlockManager:
    """Ref-counted 64-token KV block allocator with hash-based prefix caching."""

    def __init__(self, num_blocks: int):
        self._h = lib().shai_bm_create(num_blocks)
        self.num_blocks = num_blocks

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and _lib is not None:
            _lib.shai_bm_destroy(h)
            self._h = None

    @property
    def num_free(self) -> int:
        return lib().shai_bm_num_free(self._h)

    def allocate(self, n: int) -> List[int]:
        if n == 0:
            return []
        out = np.empty(n, dtype=np.int32)
        if lib().shai_bm_allocate(self._h, n, _ip(out)) != 0:
            raise MemoryError(f"out of KV blocks (need {n}, free {self.num_free})")
        return out.tolist()

    def release(self, blocks: Sequence[int]) -> None:
        if blocks:
            a = np.asarray(blocks, dtype=np.int32)
            lib().shai_bm_release(self._h, _ip(a), len(a))

    def fork(self, blocks: Sequence[int]) -> None:
        if blocks:
            a = np.asarray(blocks, dtype=np.int32)
            lib().shai_bm_fork(self._h, _ip(a), len(a))

    def register(self, block: int, content_hash: int) -> None:
        lib().shai_bm_register(self._h, int(block), ctypes.c_uint64(content_hash & 0xFFFFFFFFFFFFFFFF))

    def lookup_prefix(self, hashes: Sequence[int]) -> List[int]:
        if not hashes:
            return []
        h = np.asarray([x & 0xFFFFFFFFFFFFFFFF for x in hashes], dtype=np.uint64)
        out = np.empty(len(hashes), dtype=np.int32)
        n = lib().shai_bm_lookup_prefix(self._h, h.ctypes.data_as(_U64P), len(h), _ip(out))
        return out[:n].tolist()

    def refcount(self, block: int) -> int:
        return lib().shai_bm_refcount(self._h, int(block))

    def stats(self) -> dict:
        a = np.zeros(4, dtype=np.int64)
        lib().shai_bm_stats(self._h, a.ctypes.data_as(_I64P))
        return {"prefix_hits": int(a[0]), "prefix_queries": int(a[1]), "free": int(a[2]), "cached_free": int(a[3])}


def sched_admit(prompt_tokens: Sequence[int], free_blocks: int, running: int, max_seqs: int, token_budget: int,
                watermark_blocks: int) -> int:
    if not prompt_tokens:
        return 0
    a = np.asarray(prompt_tokens, dtype=np.int32)
    return lib().shai_sched_admit(len(a), _ip(a), free_blocks, running, max_seqs, token_budget, watermark_blocks)


def _flatten_tables(tables: Sequence[Sequence[int]]):
    offs = np.zeros(len(tables) + 1, dtype=np.int32)
    for i, t in enumerate(tables):
        offs[i + 1] = offs[i] + len(t)
    flat = np.zeros(max(1, int(offs[-1])), dtype=np.int32)
    for i, t in enumerate(tables):
        flat[offs[i]:offs[i + 1]] = t
    return flat, offs


def build_decode(ctx_before: Sequence[int], tables: Sequence[Sequence[int]], max_blocks: int):
    B = len(ctx_before)
    cb = np.asarray(ctx_before, dtype=np.int32)
    flat, offs = _flatten_tables(tables)
    pos, slots, lens = (np.empty(B, dtype=np.int32) for _ in range(3))
    bt = np.empty((B, max_blocks), dtype=np.int32)
    lib().shai_build_decode(B, _ip(cb), _ip(flat), _ip(offs), max_blocks, _ip(pos), _ip(slots), _ip(lens), _ip(bt))
    return pos, slots, lens, bt


def build_prefill(n_cached: Sequence[int], n_new: Sequence[int], tables: Sequence[Sequence[int]], S: int,
                  max_blocks: int):
    B = len(n_new)
    nc, nn = np.asarray(n_cached, dtype=np.int32), np.asarray(n_new, dtype=np.int32)
    flat, offs = _flatten_tables(tables)
    pos, slots = np.empty(B * S, dtype=np.int32), np.empty(B * S, dtype=np.int32)
    lens, qlens, last = (np.empty(B, dtype=np.int32) for _ in range(3))
    bt = np.empty((B, max_blocks), dtype=np.int32)
    lib().shai_build_prefill(B, S, _ip(nc), _ip(nn), _ip(flat), _ip(offs), max_blocks, _ip(pos), _ip(slots), _ip(lens),
                             _ip(qlens), _ip(bt), _ip(last))
    return pos, slots, lens, qlens, bt, last


def build_prefill_packed(n_cached: Sequence[int], n_new: Sequence[int], tables: Sequence[Sequence[int]],
                         max_blocks: int):
    """Varlen prefill metadata (no padding rows): positions / slots [T = sum(n_new)], per sequence ctx_lens,
    q_lens, q_start (first row), last-row index, and the padded block table [B, max_blocks]."""
    B = len(n_new)
    nc, nn = np.asarray(n_cached, dtype=np.int32), np.asarray(n_new, dtype=np.int32)
    T = int(nn.sum())
    flat, offs = _flatten_tables(tables)
    pos, slots = np.empty(max(T, 1), dtype=np.int32), np.empty(max(T, 1), dtype=np.int32)
    lens, qlens, qstart, last = (np.empty(B, dtype=np.int32) for _ in range(4))
    bt = np.empty((B, max_blocks), dtype=np.int32)
    lib().shai_build_prefill_packed(B, _ip(nc), _ip(nn), _ip(flat), _ip(offs), max_blocks, _ip(pos), _ip(slots),
                                    _ip(lens), _ip(qlens), _ip(qstart), _ip(bt), _ip(last))
    return pos[:T], slots[:T], lens, qlens, qstart, bt, last
