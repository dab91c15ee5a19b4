"""Continuous-batching LLM engine on the paged KV cache.

Replaces the vLLM ``LLM`` engine the reference builds from /vllm_config.yaml
(app/vllm_model_api.py:24-43,127-133; Neuron config with continuous batching,
buckets and on-device sampling in cova/mllama-32-11b-vllm-trn1-config.yaml) and
HF ``generate`` (app/run-llama.py:34-46, app/deepseek_model_api.py:45-57).

Per engine step (one call to :meth:`LLMEngine.step`):
  1. the native scheduler (csrc/runtime/scheduler.cpp) admits waiting prompts
     FCFS under KV-block / sequence / token budgets;
  2. admitted prompts run as one PACKED varlen prefill batch -- the step's
     sum(new tokens) rows back to back, no [B, S_max] padding, attention over
     per-sequence row offsets (prefix-cached blocks are reused via the native
     block manager's content hashes); prompts longer than ``prefill_chunk`` are
     prefilled chunk by chunk (chunked prefill), and the running batch's decode
     rows join every prefill step as one-token rows (mixed steps), so running
     sequences keep streaming while long prompts are encoded;
  3. otherwise every running sequence decodes one token -- the decode forward
     for each batch-size bucket is captured once into a HIP graph and replayed,
     with the fused RoPE / KV-write / attention kernel and the sampler inside;
  4. sampling (temperature / top-k / top-p; greedy at temperature 0) on device,
     from host-drawn uniforms (deterministic for a seed, identical on TP ranks).
With ``async_decode`` (default) steady-state decode runs one step ahead of the
host: step t+1 is enqueued (its input tokens fed from step t's output on the
device) before step t's tokens are read back, so a sequence's ``output`` grows
one ``step()`` call after its token was computed; a step past a stop token is
dropped, and steps that would pass ``max_tokens`` are never enqueued.
With TP > 1 every rank runs the same deterministic loop (SPMD); logits are
all-gathered so all ranks sample identically.
"""
from __future__ import annotations

import hashlib
import itertools
import math
import os
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from ..utils import profiling as prof
from .. import ops
from . import new_graph
from ..models.llama import (KV_BLOCK, Batch, LlamaConfig, LlamaForCausalLM, allocate_kv_cache, kv_bytes_per_block)
from ..parallel.state import tp
from ..weights import materialize


@dataclass
class SamplingParams:
    temperature: float = 0.7
    top_k: int = 50
    top_p: float = 0.9
    max_tokens: int = 128
    stop_token_ids: Optional[List[int]] = None
    ignore_eos: bool = False
    seed: Optional[int] = None


@dataclass(eq=False)  # identity semantics: membership tests must not deep-compare prompts (O(B^2))
class Sequence_:
    seq_id: int
    prompt: List[int]
    params: SamplingParams
    output: List[int] = field(default_factory=list)
    blocks: List[int] = field(default_factory=list)
    n_cached: int = 0        # tokens whose K/V are in the cache
    image: Optional[dict] = None                                 # preprocessed image (multimodal models)
    img_pos: int = -1                                            # index of <|image|> in the prompt
    cross_blocks: List[int] = field(default_factory=list)        # paged blocks holding the image K/V
    prefill_started: bool = False                                # first prefill chunk done (blocks held)
    rng_key: int = 0                                             # sampling-noise stream (seq_uniforms)
    arrival: float = field(default_factory=time.perf_counter)
    first_token_time: Optional[float] = None
    finish_time: Optional[float] = None
    finished: bool = False
    finish_reason: Optional[str] = None

    @property
    def tokens(self) -> List[int]:
        return self.prompt + self.output

    @property
    def length(self) -> int:
        return len(self.prompt) + len(self.output)

    @property
    def last_token(self) -> int:
        return self.output[-1] if self.output else self.prompt[-1]


def _mix64(x: np.ndarray) -> np.ndarray:
    """splitmix64 finaliser on uint64 arrays (wrap-around arithmetic)."""
    with np.errstate(over="ignore"):
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return x ^ (x >> np.uint64(31))


def seq_uniforms(keys: Sequence[int], positions: Sequence[int]) -> np.ndarray:
    """One U[0,1) float32 per (sequence key, absolute token position): a counter-based draw, so a sequence's
    sampling noise depends only on its key (``SamplingParams.seed`` or engine seed + sequence id) and on the
    position of the token being sampled -- not on which other sequences share the batch, on look-ahead
    steps whose tokens are dropped, or on preemption (a recomputed sequence redraws the same values)."""
    k = np.asarray(keys, dtype=np.uint64)
    p = np.asarray(positions, dtype=np.uint64)
    h = _mix64(_mix64(k) ^ p)
    return (h >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / (1 << 24))


def _chain_hash(prev: int, toks: Sequence[int]) -> int:
    h = hashlib.blake2b(digest_size=8)
    h.update(prev.to_bytes(8, "little"))
    h.update(np.asarray(toks, dtype=np.int32).tobytes())
    return int.from_bytes(h.digest(), "little") or 1


def sample(logits: torch.Tensor, temps: torch.Tensor, top_k: torch.Tensor, top_p: torch.Tensor,
           gen: Optional[torch.Generator] = None, all_greedy: Optional[bool] = None,
           uniforms: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None,
           full_vocab: Optional[bool] = None) -> torch.Tensor:
    """Temperature / top-k / top-p sampling; rows with temperature 0 are greedy (an all-greedy batch
    skips the sort / multinomial path entirely).  ``uniforms`` (one U[0,1) per row) makes the draw a
    pure function of its inputs -- what the captured decode step uses (the engine draws them on the host);
    without it they come from ``gen``.  ``out`` (int32) receives the GPU sampler's tokens in place."""
    if all_greedy:
        return logits.float().argmax(-1)
    if full_vocab is None:   # rows without a top-k in (0, 1024] sample over the whole vocabulary (torch path)
        full_vocab = bool(((top_k <= 0) | (top_k > ops.SAMPLER_MAX_K)).any()) if top_k.numel() else False
    if (logits.is_cuda and logits.dim() == 2 and not full_vocab
            and os.environ.get("SHAI_TORCH_SAMPLER", "0") != "1"):
        # fused on-device sampler (csrc/kernels/sampling.hip): top-k candidates (k <= 1024) -> top-p -> draw
        u = uniforms if uniforms is not None else torch.rand(logits.shape[0], device=logits.device, generator=gen)
        if out is not None:
            ops.sample(logits.contiguous(), temps.float().contiguous(), top_k.int().contiguous(),
                       top_p.float().contiguous(), u, out)
            return out
        out = torch.empty(logits.shape[0], dtype=torch.int32, device=logits.device)
        ops.sample(logits.contiguous(), temps.float().contiguous(), top_k.int().contiguous(),
                   top_p.float().contiguous(), u, out)
        return out.long()
    lf = logits.float()
    greedy = lf.argmax(-1)
    if all_greedy is None:
        all_greedy = bool((temps <= 0).all())
    if all_greedy:
        return greedy
    V = lf.shape[-1]
    kmax = int(top_k.max().item()) if top_k.numel() else 0
    K = V if kmax <= 0 or kmax > V or bool((top_k <= 0).any()) else kmax
    t = torch.clamp(temps, min=1e-5).unsqueeze(-1)
    vals, idx = torch.topk(lf / t, K, dim=-1)
    ar = torch.arange(K, device=lf.device).unsqueeze(0)
    kk = torch.where(top_k <= 0, torch.full_like(top_k, K), top_k).unsqueeze(-1)
    vals = vals.masked_fill(ar >= kk, float("-inf"))
    probs = torch.softmax(vals, -1)
    cum = probs.cumsum(-1)
    probs = probs.masked_fill((cum - probs) > top_p.unsqueeze(-1), 0.0)
    probs = probs / probs.sum(-1, keepdim=True)
    if uniforms is not None:  # inverse CDF at the supplied uniform (the GPU sampler's rule)
        cdf = probs.cumsum(-1)
        pick = torch.searchsorted(cdf, (uniforms.float() * cdf[:, -1]).unsqueeze(-1).contiguous(), right=True)
        pick = pick.clamp_(max=K - 1).squeeze(-1)
    else:
        pick = torch.multinomial(probs, 1, generator=gen).squeeze(-1)
    sampled = idx.gather(-1, pick.unsqueeze(-1)).squeeze(-1)
    return torch.where(temps <= 0, greedy, sampled)


class _DecodeGraph:
    """One decode step for batch bucket ``Bc`` as a single captured program (HIP graph on the GPU):
    token feedback -> model forward -> sampling -> publish tokens.

    Every per-step input (token ids, positions, KV slots, context lengths, sampling parameters, host-drawn
    uniforms, the feedback row map and the block table) lives in ONE int32 device buffer that is filled by
    ONE pinned host->device copy per step (double-buffered host side).  Sampling runs inside the graph, so a
    step's only device->host traffic is the ``Bc`` sampled token ids, copied asynchronously behind an event.

    Token feedback: row ``i`` with ``rowmap[i] >= 0`` takes its input token from row ``rowmap[i]`` of the
    previous decode step's output (``engine.last_tokens``) instead of the host id.  This is what lets the
    engine enqueue step t+1 before it has read step t's tokens back (``LLMEngine.async_decode``)."""

    NF = 9  # per-row int32 fields before the block table

    def __init__(self, engine: "LLMEngine", Bc: int, cross: bool = False, greedy: bool = False,
                 splits: Optional[int] = None, full_vocab: bool = False):
        self.Bc = Bc
        # full_vocab: some row samples with top_k <= 0 (or > 1024) -- the fused sampler keeps 1024 candidates,
        # so such steps publish the logits from the graph and sample them exactly over the whole vocabulary
        # (torch top-k / top-p path, same inverse-CDF rule at the same uniforms) after the replay
        self.full_vocab = full_vocab
        self.logits = None
        dev = engine.device
        mb = engine.max_blocks
        self.words = Bc * (self.NF + mb)
        self.dbuf = torch.zeros(self.words, dtype=torch.int32, device=dev)
        f = lambda i: self.dbuf[i * Bc:(i + 1) * Bc]
        self.ids, self.pos, self.slots, self.lens, self.topk = f(0), f(1), f(2), f(3), f(4)
        self.temps, self.topp, self.u = f(5).view(torch.float32), f(6).view(torch.float32), f(7).view(torch.float32)
        self.rowmap = f(8)
        self.bt = self.dbuf[self.NF * Bc:].view(Bc, mb)
        self.slots.fill_(-1)
        self.lens.fill_(1)
        self.rowmap.fill_(-1)
        self.toks = torch.zeros(Bc, dtype=torch.int32, device=dev)
        pin = dev.type == "cuda"
        self.host = [torch.zeros(self.words, dtype=torch.int32, pin_memory=pin) for _ in range(2)]
        self.host_np = [h.numpy() for h in self.host]
        self.host_ev = [None, None]
        self.flip = 0
        self.splits = splits if splits is not None else engine.decode_splits(Bc, 0)
        self.batch = Batch(self.ids, self.pos, self.slots, self.bt, self.lens, None, Bc, 1, False, self.splits)
        self.cross = cross
        self.greedy = greedy
        if cross:  # static image-K/V inputs of the cross-attention layers
            b = self.batch
            b.cross_bt = torch.zeros(Bc, engine.max_cross_blocks, dtype=torch.int32, device=dev)
            b.cross_lens = torch.ones(Bc, dtype=torch.int32, device=dev)
            b.cross_attn_rows = torch.zeros(Bc, dtype=torch.bool, device=dev)
            b.cross_mlp_rows = torch.zeros(Bc, dtype=torch.bool, device=dev)
            b.cross_splits = ops.decode_splits(Bc, engine.model.kv_heads_local, engine.cross_tokens)
        self.graph = None
        self.engine = engine
        if engine.use_graphs:
            # the warm-up runs publish junk tokens: keep the in-flight step's feedback tokens intact
            saved = engine.last_tokens.clone()
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(2):
                    self._program()
            torch.cuda.current_stream().wait_stream(s)
            self.graph = new_graph(dev)
            with torch.cuda.graph(self.graph):
                self._program()
            engine.last_tokens.copy_(saved)

    def _program(self):
        eng = self.engine
        ops.token_feedback(self.ids, self.rowmap, eng.last_tokens)
        logits = eng.model(self.batch, eng.kv)
        if self.full_vocab:
            self.logits = logits
            return
        if self.greedy:
            self.toks.copy_(logits.float().argmax(-1))
        elif logits.is_cuda:   # full_vocab=False: no host-side inspection of the (captured) top-k values
            sample(logits, self.temps, self.topk, self.topp, uniforms=self.u, out=self.toks, full_vocab=False)
        else:
            self.toks.copy_(sample(logits, self.temps, self.topk, self.topp, uniforms=self.u))
        eng.last_tokens[:self.Bc].copy_(self.toks)

    def launch(self, seqs, pos, slots, lens, bt, ids, rowmap, uniforms, cross=None):
        """Enqueue one decode step; returns (host int32 token view, completion event or None)."""
        B, Bc = len(seqs), self.Bc
        i = self.flip
        self.flip ^= 1
        if self.host_ev[i] is not None:  # the copy that last read this host buffer has completed
            self.host_ev[i].synchronize()
        h = self.host_np[i]
        v = lambda k: h[k * Bc:(k + 1) * Bc]
        v(0)[:B] = ids
        v(1)[:B] = pos
        v(2)[:B] = slots
        v(3)[:B] = lens
        v(4)[:B] = [s.params.top_k for s in seqs]
        v(5).view(np.float32)[:B] = [s.params.temperature for s in seqs]
        v(6).view(np.float32)[:B] = [s.params.top_p for s in seqs]
        v(7).view(np.float32)[:B] = uniforms
        v(8)[:B] = rowmap
        btv = h[self.NF * Bc:].reshape(Bc, -1)
        btv[:B] = bt
        if B < Bc:  # padding rows: no KV write, one-token context, greedy, no feedback
            v(0)[B:] = 0
            v(1)[B:] = 0
            v(2)[B:] = -1
            v(3)[B:] = 1
            v(4)[B:] = 1
            v(5).view(np.float32)[B:] = 0.0
            v(6).view(np.float32)[B:] = 1.0
            v(7).view(np.float32)[B:] = 0.0
            v(8)[B:] = -1
            btv[B:] = 0
        self.dbuf.copy_(self.host[i], non_blocking=True)
        if self.cross:
            cbt, clens, has = cross
            b = self.batch
            b.cross_bt[:B].copy_(torch.from_numpy(cbt), non_blocking=True)
            b.cross_lens[:B].copy_(torch.from_numpy(clens), non_blocking=True)
            hb = torch.from_numpy(has)
            b.cross_attn_rows[:B].copy_(hb, non_blocking=True)
            b.cross_mlp_rows[:B].copy_(hb, non_blocking=True)
            if B < Bc:
                b.cross_bt[B:].zero_()
                b.cross_lens[B:].fill_(1)
                b.cross_attn_rows[B:].fill_(False)
                b.cross_mlp_rows[B:].fill_(False)
        if self.dbuf.is_cuda:
            ev = torch.cuda.Event()
            ev.record()
            self.host_ev[i] = ev
        if self.graph is not None:
            self.graph.replay()
        else:
            self._program()
        eng = self.engine
        if self.full_vocab:   # exact full-vocabulary top-k / top-p at the same uniforms, outside the graph
            self.toks.copy_(sample(self.logits, self.temps, self.topk, self.topp, uniforms=self.u, full_vocab=True))
            eng.last_tokens[:self.Bc].copy_(self.toks)
        out = eng.tok_host[eng.tok_flip][:Bc]
        eng.tok_flip ^= 1
        out.copy_(self.toks, non_blocking=True)
        done = None
        if self.dbuf.is_cuda:
            done = torch.cuda.Event()
            done.record()
        return out, done


class _Inflight:
    """A decode step that has been enqueued but whose tokens the host has not consumed yet."""
    __slots__ = ("seqs", "toks", "event", "cross")

    def __init__(self, seqs, toks, event, cross):
        self.seqs, self.toks, self.event, self.cross = seqs, toks, event, cross


class LLMEngine:
    def __init__(self, cfg: LlamaConfig, device="cuda", model_path: Optional[str] = None, seed: int = 0,
                 max_num_seqs: int = 64, max_model_len: int = 4096, num_kv_blocks: Optional[int] = None,
                 gpu_memory_utilization: float = 0.85, prefill_token_budget: int = 8192, use_graphs: bool = True,
                 enable_prefix_caching: bool = True, prefill_chunk: Optional[int] = None,
                 quantization: Optional[str] = None, async_decode: Optional[bool] = None,
                 packed_prefill: bool = True, mixed_steps: bool = True):
        from ..models.mllama import MllamaConfig, MllamaForConditionalGeneration
        from ..runtime import BlockManager
        self.mcfg = cfg if isinstance(cfg, MllamaConfig) else None
        if self.mcfg is not None:
            cfg = self.mcfg.text
        self.cfg = cfg
        self.device = torch.device(device)
        with torch.device(self.device):
            self.model = (MllamaForConditionalGeneration(self.mcfg) if self.mcfg is not None
                          else LlamaForCausalLM(cfg))
        materialize(self.model, self.device, model_path, None, seed)
        self.model.fold_norms()  # before any graph capture (re-folded lazily after a later load)
        self.weights = self.model._shai_weights
        # vLLM-style ``quantization: fp8``: fp8 e4m3 weights + per-row scales for every TP linear
        # (after the norm fold, which rescales weight columns); decode GEMMs stream half the bytes
        self.quantization = (quantization or "").lower() or None
        if self.quantization == "fp8":
            from ..parallel.layers import quantize_fp8_
            quantize_fp8_(self.model)
        elif self.quantization not in (None, "none", "bf16"):
            raise ValueError(f"quantization={quantization!r}: supported: fp8 (weight-only e4m3) or none")
        self.max_num_seqs = max_num_seqs
        self.max_model_len = min(max_model_len, cfg.max_position_embeddings)
        self.max_blocks = (self.max_model_len + KV_BLOCK - 1) // KV_BLOCK
        self.cross_tokens = self.model.tokens_per_image if self.mcfg is not None else 0
        self.max_cross_blocks = (self.cross_tokens + KV_BLOCK - 1) // KV_BLOCK
        hk = self.model.kv_heads_local
        per_seq = self.max_blocks + self.max_cross_blocks
        if num_kv_blocks is None:
            if self.device.type == "cuda":
                free, total = torch.cuda.mem_get_info(self.device)
                budget = free - (1 - gpu_memory_utilization) * total
                num_kv_blocks = int(max(budget, 0) // kv_bytes_per_block(cfg, hk))
                num_kv_blocks = max(16, min(num_kv_blocks, max_num_seqs * per_seq + 64))
            else:
                num_kv_blocks = max_num_seqs * per_seq + 8
        self.num_kv_blocks = num_kv_blocks
        self.kv_buf, self.kv = allocate_kv_cache(cfg, hk, num_kv_blocks, self.device)
        self.bm = BlockManager(num_kv_blocks)
        self.prefill_token_budget = prefill_token_budget
        # longest prompt slice one prefill step processes (chunked prefill; SURVEY 5.7: <= 8k tokens)
        self.prefill_chunk = max(KV_BLOCK, prefill_chunk or prefill_token_budget)
        self._last_step = "decode"
        # packed varlen prefill (no [B, S_max] padding) with decode rows mixed into prefill steps (text models)
        self.packed_prefill = packed_prefill and os.environ.get("SHAI_PADDED_PREFILL", "0") != "1"
        self.mixed_steps = mixed_steps
        self.prefix_caching = enable_prefix_caching
        self.use_graphs = use_graphs and self.device.type == "cuda"
        self.waiting: List[Sequence_] = []
        self.running: List[Sequence_] = []
        self._ids = itertools.count()
        self._graphs: Dict[tuple, _DecodeGraph] = {}
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(seed)
        self.seed = int(seed)   # sampling uniforms: seq_uniforms(key, position), host-drawn (identical on TP ranks)
        # decode steps run one ahead of the host (step t+1 enqueued before step t's tokens are read back)
        if async_decode is None:
            async_decode = os.environ.get("SHAI_ASYNC_DECODE", "1") != "0"
        self.async_decode = bool(async_decode)
        self._inflight: Optional[_Inflight] = None
        bmax = 1 << max(0, math.ceil(math.log2(max(1, max_num_seqs))))
        self.last_tokens = torch.zeros(bmax, dtype=torch.int32, device=self.device)
        pin = self.device.type == "cuda"
        self.tok_host = [torch.zeros(bmax, dtype=torch.int32, pin_memory=pin) for _ in range(2)]
        self.tok_flip = 0
        self.stats = {"prefill_tokens": 0, "decode_tokens": 0, "steps": 0, "prefix_hit_tokens": 0}
        self.eos = {cfg.eos_token_id}

    def decode_splits(self, Bc: int, max_ctx: int) -> int:
        """Split-K factor of the decode attention for a batch whose longest context is ``max_ctx`` tokens:
        the chip-filling factor for short contexts (``ops.decode_splits``), raised so that no (sequence, KV
        head) workgroup walks more than ``SHAI_DECODE_SPLIT_TOKENS`` (1024) tokens when a long-context
        sequence is in the batch (one 16k-token sequence among short ones would otherwise stream its whole
        cache through 1-2 workgroups per head).  Powers of two: each value is one captured graph."""
        base = ops.decode_splits(Bc, self.model.kv_heads_local, self.max_model_len)
        per = int(os.environ.get("SHAI_DECODE_SPLIT_TOKENS", "1024"))
        need = 1
        while need < 64 and need * per < max_ctx:
            need *= 2
        return max(base, min(need, max(1, (self.max_model_len + KV_BLOCK - 1) // KV_BLOCK)))

    def warmup_graphs(self, greedy_too: bool = False) -> int:
        """Capture the decode-step HIP graph of every batch bucket (1, 2, 4, ... >= max_num_seqs) now, so no
        request pays a capture when the running batch first reaches a new bucket.  Returns how many were
        captured.  (The warm-up forwards use padding rows only: no KV-cache row is written.)"""
        if not self.use_graphs:
            return 0
        n, Bc = 0, 1
        while True:
            for greedy in ((False, True) if greedy_too else (False,)):
                key = (Bc, False, greedy, self.decode_splits(Bc, 0))
                if key not in self._graphs:
                    self._graphs[key] = _DecodeGraph(self, Bc, cross=False, greedy=greedy, splits=key[3])
                    n += 1
            if Bc >= self.max_num_seqs:
                return n
            Bc *= 2

    # ------------------------------------------------------------------ requests
    def add_request(self, prompt: Sequence[int], params: Optional[SamplingParams] = None, image=None) -> Sequence_:
        """image: PIL image / HWC uint8 array / preprocess_image() dict (multimodal models only); the prompt
        gets an ``<|image|>`` token after BOS if it has none."""
        params = params or SamplingParams()
        prompt = list(prompt)[-(self.max_model_len - 1):] or [self.cfg.bos_token_id]
        img = None
        pos = -1
        if image is not None:
            if self.mcfg is None:
                raise ValueError("this model has no vision tower; drop the image or load Llama-3.2-Vision")
            from ..models.mllama import preprocess_image
            img = image if isinstance(image, dict) else preprocess_image(image, self.mcfg.vision, self.device)
            itok = self.mcfg.image_token_index
            if itok not in prompt:
                at = 1 if prompt and prompt[0] == self.cfg.bos_token_id else 0
                prompt = prompt[:at] + [itok] + prompt[at:]
            pos = prompt.index(itok)
        sid = next(self._ids)
        key = (int(params.seed) & ((1 << 63) - 1)) | (1 << 63) if params.seed is not None else (self.seed << 32) + sid
        s = Sequence_(sid, prompt, params, image=img, img_pos=pos, rng_key=key)
        self.waiting.append(s)
        return s

    def has_work(self) -> bool:
        return bool(self.waiting or self.running or self._inflight is not None)

    def abort_all(self) -> List[Sequence_]:
        """Drop every request (after a failed step): KV blocks go back to the pool, nothing stays in flight.
        Returns the aborted sequences."""
        if self._inflight is not None and self._inflight.event is not None:
            try:
                self._inflight.event.synchronize()
            except Exception:  # the failed step's event may itself be broken
                pass
        self._inflight = None
        gone = self.waiting + self.running
        for s in gone:
            if s.blocks or s.cross_blocks:
                self._free(s)
            s.finished, s.finish_reason = True, "abort"
        self.waiting, self.running = [], []
        return gone

    # ------------------------------------------------------------------ kv blocks
    def _ensure_blocks(self, s: Sequence_, n_tokens: int) -> bool:
        need = (n_tokens + KV_BLOCK - 1) // KV_BLOCK - len(s.blocks)
        if need <= 0:
            return True
        if self.bm.num_free < need:
            return False
        s.blocks += self.bm.allocate(need)
        return True

    def _free(self, s: Sequence_):
        self.bm.release(s.blocks + s.cross_blocks)
        s.blocks = []
        s.cross_blocks = []

    def _prefix_hashes(self, toks: Sequence[int], n_full: int) -> List[int]:
        hs, h = [], 0
        for i in range(n_full):
            h = _chain_hash(h, toks[i * KV_BLOCK:(i + 1) * KV_BLOCK])
            hs.append(h)
        return hs

    # ------------------------------------------------------------------ steps
    def _admit(self) -> List[Sequence_]:
        from ..runtime import sched_admit
        if not self.waiting:
            return []
        watermark = max(1, len(self.running))
        n = sched_admit([len(s.prompt) for s in self.waiting], self.bm.num_free, len(self.running),
                        self.max_num_seqs, self.prefill_token_budget, watermark)
        if self.mcfg is not None:  # image K/V blocks are outside the native scheduler's block budget
            free, k = self.bm.num_free - watermark, 0
            for s in self.waiting[:n]:
                need = (len(s.prompt) + KV_BLOCK) // KV_BLOCK + (self.max_cross_blocks if s.image is not None else 0)
                if need > free:
                    break
                free -= need
                k += 1
            if k == 0 and n > 0 and not self.running:
                raise MemoryError("KV block pool too small for one multimodal request")
            n = k
        adm = self.waiting[:n]
        del self.waiting[:n]
        return adm

    def _prefill(self, seqs: List[Sequence_], decode_rows: Sequence[Sequence_] = ()):
        """One prefill chunk for each of ``seqs``: at most ``prefill_chunk`` new prompt tokens per sequence
        (chunked prefill -- a long prompt spans several engine steps).  The first chunk looks up cached prefix
        blocks and allocates the sequence's KV (and image) blocks; only sequences whose prompt is complete
        sample their first token.

        Text models run the step PACKED: the T = sum(new tokens) rows go back to back through every GEMM (no
        [B, S_max] padding) and attention takes per-sequence row offsets (``ops.paged_attention_varlen``).
        ``decode_rows`` -- running sequences that would otherwise wait for this prefill step -- join it as
        one-token rows (their last token against their cached context), so prefill chunks and decode share
        the step instead of alternating with it."""
        for s in seqs:
            if s.prefill_started:
                continue
            s.prefill_started = True
            s._hashes = []
            if self.prefix_caching and s.image is None:  # image prompts: K/V depend on the image, not cached
                n_full = (len(s.prompt) - 1) // KV_BLOCK
                hs = self._prefix_hashes(s.prompt, n_full)
                got = self.bm.lookup_prefix(hs)
                s.blocks = list(got)
                s.n_cached = len(got) * KV_BLOCK
                s._hashes = hs
                self.stats["prefix_hit_tokens"] += s.n_cached
            ok = self._ensure_blocks(s, len(s.prompt) + 1)
            assert ok, "scheduler admitted a prompt without blocks"
            if s.image is not None and not s.cross_blocks:
                s.cross_blocks = self.bm.allocate(self.max_cross_blocks)
                s._img_encoded = False
        packed = self.mcfg is None and self.packed_prefill
        decode_rows = [s for s in decode_rows if self._ensure_blocks(s, s.length)] if packed else []
        rows = list(seqs) + decode_rows
        n_pre = len(seqs)
        news = [min(len(s.prompt) - s.n_cached, self.prefill_chunk) for s in seqs] + [1] * len(decode_rows)
        S = max(news)
        d = self.device
        t = lambda a: torch.from_numpy(a).to(d, non_blocking=True)
        if packed:
            from ..runtime import build_prefill_packed
            pos, slots, lens, qlens, qstart, bt, last = build_prefill_packed([s.n_cached for s in rows], news,
                                                                             [s.blocks for s in rows],
                                                                             self.max_blocks)
            ids = np.concatenate([np.asarray((s.prompt if not s.output else s.tokens)[s.n_cached:s.n_cached + n],
                                             dtype=np.int32) for s, n in zip(rows, news)])
            batch = Batch(t(ids), t(pos), t(slots), t(bt), t(lens), t(qlens), len(rows), S, True, 1,
                          t(last).long(), q_start=t(qstart))
        else:
            from ..runtime import build_prefill
            pos, slots, lens, qlens, bt, last = build_prefill([s.n_cached for s in seqs], news,
                                                              [s.blocks for s in seqs], S, self.max_blocks)
            ids = np.zeros(len(seqs) * S, dtype=np.int32)
            for i, (s, n) in enumerate(zip(seqs, news)):
                ids[i * S:i * S + n] = s.prompt[s.n_cached:s.n_cached + n]
            batch = Batch(t(ids), t(pos), t(slots), t(bt), t(lens), t(qlens), len(seqs), S, True, 1, t(last).long())
        if any(s.cross_blocks for s in seqs):
            fresh = [s for s in seqs if s.cross_blocks and not s._img_encoded]
            if fresh:
                self._encode_images(fresh)
                for s in fresh:
                    s._img_encoded = True
            self._attach_cross_prefill(batch, seqs, S, news)
        logits = self.model(batch, self.kv)
        self.stats["prefill_tokens"] += int(sum(news[:n_pre]))
        self.stats["decode_tokens"] += len(decode_rows)
        done = []
        for i, (s, n) in enumerate(zip(rows, news)):
            s.n_cached += n
            if i >= n_pre:       # decode row: always samples its next token
                done.append(i)
                continue
            if s.n_cached < len(s.prompt):
                continue
            done.append(i)
            if self.prefix_caching:
                for j, h in enumerate(s._hashes):
                    self.bm.register(s.blocks[j], h)
        if done:
            sel = logits if len(done) == len(rows) else logits.index_select(0, torch.tensor(done, device=d))
            self._sample_and_append([rows[i] for i in done], sel)

    # ------------------------------------------------------------------ images (multimodal models)
    def _encode_images(self, seqs: List[Sequence_]):
        """Vision tower + projector for every new image, then each cross layer's K/V into the sequence's
        image blocks (once per request; decode steps only read them)."""
        d = self.device
        px = torch.stack([s.image["pixel_values"].to(d) for s in seqs])
        ar = torch.tensor([s.image["aspect_ratio_id"] for s in seqs], device=d)
        states = self.model.encode_images(px, ar, [s.image["num_tiles"] for s in seqs])
        nv = np.arange(self.cross_tokens)
        slots = np.concatenate([np.asarray(s.cross_blocks, np.int64)[nv // KV_BLOCK] * KV_BLOCK + nv % KV_BLOCK
                                for s in seqs]).astype(np.int32)
        self.model.write_cross_kv(states.reshape(-1, states.shape[-1]), self.kv, torch.from_numpy(slots).to(d))

    def _cross_tables(self, seqs: List[Sequence_]):
        B, P = len(seqs), self.mcfg.vision.num_patches
        cbt = np.zeros((B, self.max_cross_blocks), np.int32)
        clens = np.ones(B, np.int32)
        has = np.zeros(B, bool)
        for i, s in enumerate(seqs):
            if s.cross_blocks:
                cbt[i] = s.cross_blocks
                clens[i] = s.image["num_tiles"] * P
                has[i] = True
        return cbt, clens, has

    def _attach_cross_prefill(self, batch: Batch, seqs: List[Sequence_], S: int, news: List[int]):
        cbt, clens, has = self._cross_tables(seqs)
        full = np.where(has, self.cross_tokens, 1).astype(np.int32)
        # rows of this chunk that lie before <|image|>
        pre = np.asarray([min(n, max(0, s.img_pos - s.n_cached)) if s.cross_blocks else 0
                          for s, n in zip(seqs, news)], np.int32)
        pre_rows = (np.arange(S)[None, :] < pre[:, None]) & has[:, None]
        attn_rows = np.repeat(has[:, None], S, axis=1)
        d = self.device
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(d, non_blocking=True)
        batch.cross_bt, batch.cross_lens, batch.cross_full_lens = t(cbt), t(clens), t(full)
        batch.cross_pre_lens = t(pre) if pre.any() else None
        batch.cross_pre_rows = t(pre_rows.reshape(-1))
        batch.cross_attn_rows = t(attn_rows.reshape(-1))
        batch.cross_mlp_rows = t((attn_rows & ~pre_rows).reshape(-1))

    def _decode(self, seqs: List[Sequence_]) -> Optional[_Inflight]:
        """Enqueue one decode step of ``seqs`` (host-known token ids); the tokens are consumed by
        :meth:`_finish_decode`."""
        for s in seqs:
            if not self._ensure_blocks(s, s.length):
                # preempt (recompute later): free blocks, requeue at the front
                self._free(s)
                s.n_cached = 0
                s.prefill_started = False
                s.prompt = s.prompt + s.output
                s.output = []
                self.running.remove(s)
                self.waiting.insert(0, s)
        running = set(map(id, self.running))
        seqs = [s for s in seqs if id(s) in running]
        if not seqs:
            return None
        return self._launch(seqs, [s.length - 1 for s in seqs], [s.last_token for s in seqs], [-1] * len(seqs))

    def _launch(self, seqs, ctx_before, ids, rowmap) -> _Inflight:
        from ..runtime import build_decode
        B = len(seqs)
        pos, slots, lens, bt = build_decode(ctx_before, [s.blocks for s in seqs], self.max_blocks)
        Bc = 1 << max(0, math.ceil(math.log2(B)))
        cross = self._cross_tables(seqs) if any(s.cross_blocks for s in seqs) else None
        greedy = all(s.params.temperature <= 0 for s in seqs)
        splits = self.decode_splits(Bc, int(lens.max()) if B else 0)
        full = (not greedy) and any(s.params.temperature > 0 and not 0 < s.params.top_k <= ops.SAMPLER_MAX_K
                                    for s in seqs)
        key = (Bc, cross is not None, greedy, splits) + ((True,) if full else ())
        g = self._graphs.get(key)
        if g is None:
            g = self._graphs[key] = _DecodeGraph(self, Bc, cross=cross is not None, greedy=greedy, splits=splits,
                                                 full_vocab=full)
        # noise for the token each row samples, at absolute position ctx_before + 1
        u = (seq_uniforms([s.rng_key for s in seqs], [c + 1 for c in ctx_before]) if not greedy
             else np.zeros(B, np.float32))
        toks, ev = g.launch(seqs, pos, slots, lens, bt, ids, rowmap, u, cross)
        self.stats["decode_tokens"] += B
        return _Inflight(seqs, toks, ev, cross is not None)

    def _finish_decode(self, h: _Inflight):
        """Consume an enqueued decode step's tokens (rows of sequences that finished meanwhile -- the
        look-ahead step past an EOS -- are dropped)."""
        if h.event is not None:
            h.event.synchronize()
        toks = h.toks[:len(h.seqs)].tolist()
        live = [(s, t) for s, t in zip(h.seqs, toks) if not s.finished]
        for s, _ in live:
            s.n_cached = s.length
        self._append([s for s, _ in live], [t for _, t in live])

    def _lookahead(self, prev: _Inflight) -> Optional[_Inflight]:
        """Enqueue the next decode step before ``prev``'s tokens are read back, feeding ``prev``'s sampled
        tokens on the device.  Only in steady-state decode (nothing waiting, no prefill chunk pending, no
        image cross-attention); sequences that ``prev`` completes by length are left out, and a sequence
        that ``prev`` ends by a stop token produces one extra token that :meth:`_finish_decode` drops."""
        if not self.async_decode or prev.cross or self.waiting:
            return None
        if any(s.n_cached < len(s.prompt) for s in self.running):
            return None
        in_prev = set(map(id, prev.seqs))
        if any(id(s) not in in_prev for s in self.running if not s.finished):
            return None
        nxt, rows = [], []
        for i, s in enumerate(prev.seqs):
            if s.finished:
                continue
            n_out = len(s.output) + 1           # after prev's token
            if n_out >= s.params.max_tokens or s.length + 1 >= self.max_model_len:
                continue
            nxt.append(s)
            rows.append(i)
        if not nxt:
            return None
        for s in nxt:  # blocks for the token fed at position s.length (prev's output)
            if not self._ensure_blocks(s, s.length + 1):
                return None
        return self._launch(nxt, [s.length for s in nxt], [0] * len(nxt), rows)

    def _sample_and_append(self, seqs, logits):
        d = self.device
        temps = torch.tensor([s.params.temperature for s in seqs], dtype=torch.float32, device=d)
        tk = torch.tensor([s.params.top_k for s in seqs], dtype=torch.int64, device=d)
        tpp = torch.tensor([s.params.top_p for s in seqs], dtype=torch.float32, device=d)
        greedy = all(s.params.temperature <= 0 for s in seqs)
        u = None if greedy else torch.from_numpy(seq_uniforms([s.rng_key for s in seqs],
                                                              [s.length for s in seqs])).to(d)
        toks = sample(logits, temps, tk, tpp, self.gen, all_greedy=greedy, uniforms=u).tolist()
        self._append(seqs, toks)

    def _append(self, seqs, toks):
        now = time.perf_counter()
        for s, tok in zip(seqs, toks):
            s.output.append(int(tok))
            if s.first_token_time is None:
                s.first_token_time = now
            stop = set(s.params.stop_token_ids or []) | (set() if s.params.ignore_eos else self.eos)
            if tok in stop:
                s.finished, s.finish_reason = True, "stop"
            elif len(s.output) >= s.params.max_tokens or s.length >= self.max_model_len:
                s.finished, s.finish_reason = True, "length"
            if s.finished:
                s.finish_time = now

    def _reap(self) -> List[Sequence_]:
        done = [s for s in self.running if s.finished]
        if done:
            fin = set(map(id, done))
            for s in done:
                self._free(s)
            self.running = [s for s in self.running if id(s) not in fin]
        return done

    def step(self) -> List[Sequence_]:
        """Run one engine iteration; returns sequences that finished in it."""
        self.stats["steps"] += 1
        prev = self._inflight
        if prev is not None:
            self._inflight = self._lookahead(prev)   # step t+1 enqueued while step t is on the GPU
            self._finish_decode(prev)
            if self._inflight is not None:
                return self._reap()
        adm = self._admit()
        pending = [s for s in self.running if s.n_cached < len(s.prompt)]     # mid chunked prefill
        decodable = [s for s in self.running if s.n_cached >= len(s.prompt) and not s.finished]
        mix = self.mcfg is None and self.packed_prefill and self.mixed_steps
        # new prompts and remaining prefill chunks run as packed prefill steps that the running batch's decode
        # rows join (mixed steps); without mixing (multimodal models) they alternate with decode steps
        if adm or (pending and (mix or not decodable or self._last_step != "prefill")):
            self.running += adm
            with prof.range_("llm_prefill"):
                self._prefill(pending + adm, decodable if mix else ())
            self._last_step = "prefill"
        elif decodable:
            with prof.range_("llm_decode"):
                h = self._decode(decodable)
            if h is not None:
                if self.async_decode and not h.cross:
                    self._inflight = h   # tokens consumed by the next step (after it enqueues its own)
                else:
                    self._finish_decode(h)
            self._last_step = "decode"
        if tp().size > 1:  # a timed-out xGMI peer collective leaves partial sums: fail the step loudly
            from ..parallel.comm import raise_if_p2p_error
            raise_if_p2p_error()
        return self._reap()

    @torch.inference_mode()
    def generate(self, prompts: Sequence[Sequence[int]], params: Optional[SamplingParams] = None) -> List[Sequence_]:
        seqs = [self.add_request(p, params) for p in prompts]
        while any(not s.finished for s in seqs):
            self.step()
        if self._inflight is not None and not any(not s.finished for s in self._inflight.seqs):
            self.step()  # a look-ahead step past the last stop token: retire it (its tokens are dropped)
        return seqs


# ---------------------------------------------------------------------- helpers
def smoke_llm(device="cuda:0"):
    eng = LLMEngine(LlamaConfig.tiny(), device=device, max_num_seqs=4, max_model_len=256)
    out = eng.generate([[1, 5, 9, 200], list(range(3, 90))], SamplingParams(max_tokens=4, temperature=0.0,
                                                                            ignore_eos=True))
    assert all(len(s.output) == 4 for s in out)
    return out


def bench_decode_throughput(args, rank, world):
    """Mistral-7B bf16, ``args.tp``-way tensor parallel (default: all ``world`` GPUs), world / tp data-parallel
    replicas: each replica generates gen_len tokens for a batch of prompt_len-token prompts; tokens/s is the
    sum over replicas."""
    from ..parallel.state import init_distributed
    tpd = int(getattr(args, "tp", None) or world)
    assert world % tpd == 0, (world, tpd)
    replicas = world // tpd
    init_distributed(tp_size=tpd)
    name = getattr(args, "llm_model", None) or "mistral_7b"
    cfg = {"mistral_7b": LlamaConfig.mistral_7b, "llama3_8b": LlamaConfig.llama3_8b,
           "deepseek_r1_distill_70b": LlamaConfig.deepseek_r1_distill_70b}[name]()
    B, P, G = args.batch, args.prompt_len, args.gen_len
    quant = getattr(args, "quantization", None)
    eng = LLMEngine(cfg, device=f"cuda:{torch.cuda.current_device()}", max_num_seqs=max(B, 1),
                    max_model_len=P + G + 64, enable_prefix_caching=False, quantization=quant)
    params = SamplingParams(temperature=0.7, top_k=50, top_p=0.9, max_tokens=G, ignore_eos=True)
    rng = np.random.default_rng(0)
    prompts = lambda: [rng.integers(10, cfg.vocab_size - 10, P).tolist() for _ in range(B)]
    for _ in range(max(1, args.warmup)):
        eng.generate(prompts(), params)
    import torch.distributed as dist
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    ttft, tpot = [], []
    for _ in range(args.steps):
        out = eng.generate(prompts(), params)
        for s in out:
            ttft.append(s.first_token_time - s.arrival)
            tpot.append((s.finish_time - s.first_token_time) / max(1, len(s.output) - 1))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    toks = B * G * args.steps * replicas
    label = {"mistral_7b": "Mistral-7B", "llama3_8b": "Llama-3-8B",
             "deepseek_r1_distill_70b": "DeepSeek-R1-Distill-Llama-70B"}[name]
    hf = {"mistral_7b": "mistralai/Mistral-7B-Instruct-v0.3", "llama3_8b": "meta-llama/Meta-Llama-3-8B-Instruct",
          "deepseek_r1_distill_70b": "deepseek-ai/DeepSeek-R1-Distill-Llama-70B"}[name]
    return {
        "metric": (f"{label} output tokens/sec (fp8 e4m3 weights, bf16 activations, continuous batching)"
                   if quant == "fp8" else f"{label} output tokens/sec (bf16, continuous batching)"),
        "value": round(toks / el, 2), "unit": "tokens/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(1000 * el / args.steps, 2), "higher_is_better": True,
        "scaling": "strong" if replicas == 1 else "weak", "vs_baseline": None, "dtype": "fp8w-bf16a" if quant == "fp8" else "bf16",
        "data": "synthetic prompts, random-init weights",
        "config": {"model": f"{hf} (architecture)", "global_batch": B * replicas,
                   "seq_len": P + G, "prompt_len": P, "gen_len": G,
                   "parallelism": (f"dp{replicas}x" if replicas > 1 else "") + f"tp{tpd}"},
        "p50_ttft_ms": round(1000 * float(np.median(ttft)), 2), "p50_tpot_ms": round(1000 * float(np.median(tpot)), 3),
    }


# ---------------------------------------------------------------------- online service
def engine_step(engine: LLMEngine, adds) -> tuple:
    """Add ``adds`` = [(token ids, SamplingParams, image or None), ...] to ``engine`` and run one step.

    The unit of work of :class:`LLMService` -- and, at TP > 1, exactly what every follower rank executes
    for each STEP message the leader broadcasts (serving/tp.py), so all ranks make identical scheduling
    and sampling decisions and their collectives line up.  Returns (per-add Sequence_ or exception,
    finished sequences, step exception or None); a failed step aborts every request (KV blocks freed)."""
    added = []
    for ids, params, image in adds:
        try:
            added.append(engine.add_request(ids, params, image=image))
        except Exception as e:  # bad request (e.g. an image for a text-only model)
            added.append(e)
    if not engine.has_work():
        return added, [], None
    try:
        with torch.inference_mode():
            return added, engine.step(), None
    except Exception as e:  # noqa: BLE001
        engine.abort_all()
        return added, [], e


class LLMService:
    """Thread-safe front end: a dedicated engine thread runs continuous batching;
    callers submit prompts (text or ids) and wait on futures.

    Replaces the reference's offline ``LLM.generate`` per HTTP request
    (app/vllm_model_api.py:38-43), so concurrent requests share decode steps.

    ``channel`` (TP > 1, rank 0): before every engine step the requests admitted since the previous step are
    broadcast to the follower ranks (serving/tp.py), which run the same :func:`engine_step`.
    ``live``: engine liveness for ``/health`` (a step that never returns turns the replica unhealthy)."""

    def __init__(self, engine: LLMEngine, tokenizer=None, channel=None):
        import queue
        import threading
        from ..utils.liveness import Liveness, register
        self.engine = engine
        self.tokenizer = tokenizer
        self.channel = channel
        self.live = register(Liveness())
        self._q: "queue.Queue" = queue.Queue()
        self._futs = {}
        self._t = threading.Thread(target=self._loop, name="llm-engine", daemon=True)
        self._t.start()

    def _loop(self):
        import queue
        from ..serving.tp import STEP
        while True:
            items = []
            try:
                block = not self.engine.has_work()
                while True:
                    items.append(self._q.get(block=block, timeout=None if block else 0))
                    block = False
            except queue.Empty:
                pass
            adds = [(ids, params, image) for ids, params, _, image in items]
            if self.channel is not None:
                self.channel.send(STEP, adds)
            added, done, err = engine_step(self.engine, adds)
            for (_, _, fut, _), s in zip(items, added):
                if isinstance(s, Exception):
                    fut.set_exception(s)
                else:
                    self._futs[s.seq_id] = (s, fut)
            if err is not None:  # fail every in-flight request
                for sid, (s, fut) in list(self._futs.items()):
                    if not fut.done():
                        fut.set_exception(err)
                self._futs.clear()
            for s in done:
                ent = self._futs.pop(s.seq_id, None)
                if ent is not None:
                    ent[1].set_result(s)
            self.live.progress(still_pending=self.engine.has_work() or not self._q.empty())

    def submit_ids(self, ids, params: SamplingParams, image=None):
        from concurrent.futures import Future
        f = Future()
        if image is not None and self.channel is not None:
            image = np.asarray(image.convert("RGB") if hasattr(image, "convert") else image, dtype=np.uint8)
        self.live.work_pending()
        self._q.put((list(ids), params, f, image))
        return f

    @property
    def multimodal(self) -> bool:
        return self.engine.mcfg is not None

    def encode(self, text: str):
        if self.tokenizer is None:
            raise RuntimeError("no tokenizer")
        enc = self.tokenizer(text, padding="longest", truncation=True, max_length=self.engine.max_model_len - 1)
        ids = enc["input_ids"]
        ids = ids[0] if hasattr(ids, "dim") and ids.dim() == 2 else ids
        return [int(i) for i in (ids.tolist() if hasattr(ids, "tolist") else ids)]

    def generate_text(self, prompt: str, params: SamplingParams, timeout: Optional[float] = None, image=None):
        t0 = time.time()
        s = self.submit_ids(self.encode(prompt), params, image).result(timeout)
        text = self.tokenizer.decode(s.output, skip_special_tokens=True)
        return text, time.time() - t0, s


def llama_config_for(model_id: str, model_path: Optional[str] = None, size: str = "") -> LlamaConfig:
    import json
    from ..models.mllama import MllamaConfig
    if model_path and os.path.exists(os.path.join(model_path, "config.json")):
        with open(os.path.join(model_path, "config.json")) as f:
            d = json.load(f)
        if "vision_config" in d and "text_config" in d:
            return MllamaConfig.from_hf(d)
        d = d.get("text_config", d)
        return LlamaConfig.from_hf(d)
    m = (model_id or "").lower()
    vision = "vision" in m or "mllama" in m
    if size == "tiny":
        return MllamaConfig.tiny() if vision else LlamaConfig.tiny()
    if vision:
        return MllamaConfig.llama32_11b_vision()
    if "70b" in m or "deepseek" in m:
        return LlamaConfig.deepseek_r1_distill_70b() if "deepseek" in m else LlamaConfig.llama3_70b()
    if "llama" in m:
        return LlamaConfig.llama3_8b()
    return LlamaConfig.mistral_7b()
