"""Stable Diffusion 2.1 text-to-image engine.

Replaces diffusers' ``StableDiffusionPipeline`` as driven by app/run-sd.py:104-146
(and optimum-neuron's NEFF pipeline, app/compile-sd2.py:16-20).  Differences
that matter on MI355X:

* Whole UNet step captured once per (batch, resolution) bucket into a HIP
  graph (``torch.cuda.CUDAGraph`` == hipGraph on ROCm) and replayed for every
  denoising step: one host launch per step instead of ~1000 kernel launches.
  The reference explicitly runs ``max-autotune-no-cudagraphs``.
* Classifier-free guidance is batched (uncond+cond in one UNet pass) and the
  guidance combine + DDIM update is ONE fused kernel (``ops.sched_step``).
* Cross-attention K/V are projected once per request, not once per step.
* Requests can be batched (several prompts per UNet pass) by the serving layer.
"""
from __future__ import annotations

import time
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .. import ops
from . import new_graph
from ..models.clip import CLIPTextConfig, CLIPTextModel
from ..models.unet2d import UNet2DConditionModel, UNetConfig
from ..models.vae import AutoencoderKLDecoder, VAEConfig
from ..schedulers import DDIMScheduler
from ..tokenizers import load_tokenizer
from ..utils import profiling as prof
from ..weights import materialize


@dataclass
class SDConfig:
    text: CLIPTextConfig
    unet: UNetConfig
    vae: VAEConfig
    prediction_type: str = "v_prediction"   # stabilityai/stable-diffusion-2-1 (768-v); -base is "epsilon"
    height: int = 512
    width: int = 512

    @staticmethod
    def sd21(prediction_type="v_prediction", height=512, width=512):
        return SDConfig(CLIPTextConfig.sd21(), UNetConfig.sd21(), VAEConfig.sd21(), prediction_type, height, width)

    @staticmethod
    def tiny():
        return SDConfig(CLIPTextConfig(vocab_size=1000, hidden_size=64, intermediate_size=128, num_hidden_layers=1,
                                       num_attention_heads=1, bos_token_id=998, eos_token_id=999),
                        UNetConfig.tiny(), VAEConfig.tiny(), "epsilon", 64, 64)


class _UNetGraph:
    """HIP-graph-captured UNet forward for one (batch, latent HxW) bucket.  ``per_row_t``: the timestep input is
    one value per CFG row ([2B], step-level batching) instead of one for the whole batch.  ``pool``: a graph
    memory pool shared with the other buckets (they are never replayed concurrently)."""

    def __init__(self, unet: UNet2DConditionModel, B: int, h: int, w: int, ctx_len: int, ctx_shapes, device,
                 per_row_t: bool = False, pool=None):
        self.unet = unet
        self.lat = torch.zeros(B, h, w, unet.cfg.in_channels, dtype=torch.bfloat16, device=device)
        self.t = torch.zeros(2 * B if per_row_t else 1, dtype=torch.float32, device=device)
        self.kv = [torch.zeros(s, dtype=torch.bfloat16, device=device) for s in ctx_shapes]
        self.graph = new_graph(device)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                self._fwd()
        torch.cuda.current_stream().wait_stream(s)
        with torch.cuda.graph(self.graph, pool=pool):
            self.out = self._fwd()

    def _fwd(self):
        x = torch.cat([self.lat, self.lat], 0)
        return self.unet(x, self.t, self.kv)

    def run(self, t: float) -> torch.Tensor:
        self.t.fill_(t)
        self.graph.replay()
        return self.out

    def run_rows(self) -> torch.Tensor:
        """Replay with the per-row timesteps already in ``self.t``."""
        self.graph.replay()
        return self.out


class StableDiffusionEngine:
    def __init__(self, cfg: Optional[SDConfig] = None, device="cuda", model_path: Optional[str] = None, seed: int = 0,
                 use_graphs: bool = True):
        self.cfg = cfg or SDConfig.sd21()
        self.device = torch.device(device)
        with torch.device(self.device):
            self.text_encoder = CLIPTextModel(self.cfg.text)
            self.unet = UNet2DConditionModel(self.cfg.unet)
            self.vae = AutoencoderKLDecoder(self.cfg.vae)
        materialize(self.text_encoder, self.device, model_path, "text_encoder", seed)
        materialize(self.unet, self.device, model_path, "unet", seed + 1)
        materialize(self.vae, self.device, model_path, "vae", seed + 2)
        self.weights = self.unet._shai_weights
        tc = self.cfg.text
        self.tokenizer = load_tokenizer(model_path, subfolder="tokenizer", vocab_size=tc.vocab_size,
                                        bos_id=tc.bos_token_id, eos_id=tc.eos_token_id, pad_id=tc.pad_token_id,
                                        model_max_length=tc.max_position_embeddings)
        self.scheduler = DDIMScheduler(prediction_type=self.cfg.prediction_type)
        self.use_graphs = use_graphs and self.device.type == "cuda"
        self._graphs: Dict[Tuple[int, int, int], _UNetGraph] = {}
        self.unet.build_temb_bank()

    # ------------------------------------------------------------------ pieces
    @torch.no_grad()
    def encode_prompts(self, prompts: Sequence[str], negative: Optional[Sequence[str]] = None) -> torch.Tensor:
        neg = list(negative) if negative is not None else [""] * len(prompts)
        toks = self.tokenizer(neg + list(prompts), max_length=self.cfg.text.max_position_embeddings,
                              padding="max_length", truncation=True, return_tensors="pt")
        ids = toks["input_ids"].to(self.device)
        return self.text_encoder(ids)  # [2B, 77, d] (uncond first)

    def _graph_for(self, B, h, w, ctx_kv) -> _UNetGraph:
        key = (B, h, w)
        g = self._graphs.get(key)
        if g is None:
            g = _UNetGraph(self.unet, B, h, w, ctx_kv[0].shape[1], [t.shape for t in ctx_kv], self.device)
            self._graphs[key] = g
        return g

    @torch.no_grad()
    def generate(self, prompts: Sequence[str], num_inference_steps: int = 50, guidance_scale: float = 7.5,
                 height: Optional[int] = None, width: Optional[int] = None, seed: Optional[int] = None,
                 negative_prompts: Optional[Sequence[str]] = None, output: str = "uint8") -> torch.Tensor:
        """Returns NHWC images: uint8 [B, H, W, 3] on the host (output='uint8') or the
        decoder's bf16 output on device (output='tensor')."""
        H = height or self.cfg.height
        W = width or self.cfg.width
        B = len(prompts)
        h, w = H // 8, W // 8
        with prof.profile_session("sd_generate"):
            return self._generate(prompts, negative_prompts, num_inference_steps, guidance_scale, B, h, w, seed,
                                  output)

    def _generate(self, prompts, negative_prompts, num_inference_steps, guidance_scale, B, h, w, seed, output):
        with prof.range_("text_encode"):
            ctx = self.encode_prompts(prompts, negative_prompts)
            ctx_kv = self.unet.context_kv(ctx)
        gen = torch.Generator(device=self.device)
        gen.manual_seed(int(seed) if seed is not None else int(time.time_ns() % (2 ** 31)))
        lat = torch.randn(B, h, w, self.cfg.unet.in_channels, generator=gen, device=self.device,
                          dtype=torch.float32).mul_(self.scheduler.init_noise_sigma).to(torch.bfloat16)
        steps = self.scheduler.steps(num_inference_steps)
        if self.use_graphs:
            g = self._graph_for(B, h, w, ctx_kv)
            for dst, src in zip(g.kv, ctx_kv):
                dst.copy_(src)
            g.lat.copy_(lat)
            lat = g.lat
            for sp in steps:
                with prof.range_("unet_step"):
                    out = g.run(sp.t)
                ops.sched_step(out, lat, True, guidance_scale, self.scheduler.pred_type, sp.a_t, sp.a_prev)
        else:
            for sp in steps:
                t = torch.full((1,), sp.t, dtype=torch.float32, device=self.device)
                out = self.unet(torch.cat([lat, lat], 0), t, ctx_kv)
                ops.sched_step(out, lat, True, guidance_scale, self.scheduler.pred_type, sp.a_t, sp.a_prev)
        with prof.range_("vae_decode"):
            img = self.vae(lat)
        if output == "tensor":
            return img
        return AutoencoderKLDecoder.to_uint8(img).cpu()

    def __call__(self, prompt, num_inference_steps: int = 50, **kw):
        prompts = [prompt] if isinstance(prompt, str) else list(prompt)
        return self.generate(prompts, num_inference_steps, **kw)


@dataclass(eq=False)
class DiffusionRequest:
    """One txt2img request inside a :class:`StepBatcher`: its own schedule and step index."""
    prompt: str
    steps: list
    seed: int
    negative: str = ""
    i: int = 0                      # index of the next denoising step
    image: Optional[torch.Tensor] = None
    done: bool = False
    arrival: float = 0.0
    finish_time: Optional[float] = None


MAX_INFERENCE_STEPS = 1000   # the DDIM training schedule length: more steps than timesteps is meaningless


def validate_request(prompt, num_inference_steps) -> None:
    """Reject a request that cannot run before it touches shared batch state: a non-string prompt would fail the
    text encoder for every request regrouped with it, and a step count < 1 divides by zero in the schedule."""
    if not isinstance(prompt, str):
        raise ValueError(f"prompt must be a string, got {type(prompt).__name__}")
    try:
        n = int(num_inference_steps)
    except (TypeError, ValueError):
        raise ValueError(f"num_inference_steps must be an integer, got {num_inference_steps!r}") from None
    if not 1 <= n <= MAX_INFERENCE_STEPS:
        raise ValueError(f"num_inference_steps must be in [1, {MAX_INFERENCE_STEPS}], got {n}")


class StepBatcher:
    """Step-level (continuous) batching for SD2.1: a request joins the running batch at the NEXT denoising-step
    boundary instead of waiting for the whole current batch (50 steps) to finish, and leaves it as soon as its
    own schedule ends.  Every row carries its own timestep (the UNet takes a [2B] timestep vector, the time
    embedding is added per image in the conv epilogues) and its own DDIM coefficients (``ops.sched_step_rows``).

    Rows 0..n-1 of the current bucket's static buffers hold the n active requests (latents + their CFG
    cross-attention K/V); a bucket is n itself up to 16, then n rounded up to a multiple of 8 (idle rows keep
    a_t < 0 and are never updated); its UNet step is one HIP-graph replay, and all buckets share one graph
    memory pool.  When the
    membership changes the state rows are gathered into the new bucket's buffers.  Finished rows are decoded
    by the VAE in one batch.  The reference has no cross-request batching at all (run-sd.py:137-142)."""

    VAE_MAX_BATCH = 8

    def __init__(self, engine: "StableDiffusionEngine", max_batch: int = 32, guidance_scale: float = 7.5,
                 height: Optional[int] = None, width: Optional[int] = None):
        self.eng = engine
        self.max_batch = max_batch
        self.guidance = guidance_scale
        H, W = height or engine.cfg.height, width or engine.cfg.width
        self.h, self.w = H // 8, W // 8
        self.waiting: List[DiffusionRequest] = []
        self.active: List[DiffusionRequest] = []
        self.buf = None                 # current bucket: _UNetGraph (GPU) or _Rows (CPU / no graphs)
        self._graphs: Dict[int, object] = {}
        self._pool = torch.cuda.graph_pool_handle() if engine.use_graphs else None
        self._kv_shapes1 = None         # per-layer K/V shapes for ONE CFG pair (2 rows)
        self.stats = {"steps": 0, "rows": 0, "joined_mid_batch": 0}

    # ------------------------------------------------------------------ requests
    def add(self, prompt: str, num_inference_steps: int = 50, seed: Optional[int] = None,
            negative: str = "") -> DiffusionRequest:
        validate_request(prompt, num_inference_steps)
        seed = int(seed) if seed is not None else int(time.time_ns() % (2 ** 31))
        r = DiffusionRequest(prompt, self.eng.scheduler.steps(num_inference_steps), seed, negative,
                             arrival=time.perf_counter())
        self.waiting.append(r)
        return r

    def has_work(self) -> bool:
        return bool(self.waiting) or any(not r.done for r in self.active)

    @staticmethod
    def bucket(n: int) -> int:
        """Rows the step runs for n active requests: exact up to 16 (small batches are latency-critical and a
        padded row costs a whole image of UNet work), then multiples of 8."""
        return n if n <= 16 else (n + 7) // 8 * 8

    def _buffers(self, Bc: int, kv_shapes):
        if Bc not in self._graphs:
            if self.eng.use_graphs:
                self._graphs[Bc] = _UNetGraph(self.eng.unet, Bc, self.h, self.w, 77, kv_shapes, self.eng.device,
                                              per_row_t=True, pool=self._pool)
            else:
                self._graphs[Bc] = _Rows(self.eng.unet, Bc, self.h, self.w, kv_shapes, self.eng.device)
        return self._graphs[Bc]

    def warmup(self, buckets: Optional[Sequence[int]] = None) -> int:
        """Capture the step graph of every bucket (1, 2, 4, ... max_batch) before serving."""
        if self._kv_shapes1 is None:
            self._kv_shapes1 = [t.shape[1:] for t in self.eng.unet.context_kv(self.eng.encode_prompts([""]))]
        n = 0
        for Bc in buckets or sorted({self.bucket(k) for k in range(1, self.max_batch + 1)}):
            if Bc <= self.bucket(self.max_batch) and Bc not in self._graphs:
                self._buffers(Bc, [(2 * Bc,) + tuple(s) for s in self._kv_shapes1])
                n += 1
        # the VAE decodes every batch of finishing rows (1 .. VAE_MAX_BATCH): tune its convs for each size
        # now, not inside a request
        z = torch.zeros(1, self.h, self.w, self.eng.cfg.unet.in_channels, dtype=torch.bfloat16,
                        device=self.eng.device)
        for k in range(1, min(self.VAE_MAX_BATCH, self.max_batch) + 1):
            self.eng.vae(z.expand(k, -1, -1, -1).contiguous())
        # and the text encoder / cross-attention K/V for every admission size
        for k in range(1, min(self.VAE_MAX_BATCH, self.max_batch) + 1):
            self.eng.unet.context_kv(self.eng.encode_prompts([""] * k))
        return n

    # ------------------------------------------------------------------ one step
    @torch.no_grad()
    def step(self) -> List[DiffusionRequest]:
        """Admit waiting requests, run ONE denoising step for every active request, retire the finished ones
        (VAE-decoded).  Returns the requests finished in this step."""
        eng, dev = self.eng, self.eng.device
        keep = [r for r in self.active if not r.done]
        room = self.max_batch - len(keep)
        new = self.waiting[:max(0, room)]
        del self.waiting[:len(new)]
        if keep and new:
            self.stats["joined_mid_batch"] += len(new)
        rows = keep + new
        if not rows:
            self.active = []
            return []
        if new or len(keep) != len(self.active) or self.buf is None:
            self._regroup(keep, new)
        n = len(rows)
        buf, Bc = self.buf, self.buf.lat.shape[0]
        tv = np.zeros(2 * Bc, np.float32)
        pv = np.full((Bc, 3), -1.0, np.float32)
        for j, r in enumerate(rows):
            sp = r.steps[r.i]
            tv[j] = tv[Bc + j] = sp.t
            pv[j] = (sp.a_t, sp.a_prev, sp.dt)
        buf.t.copy_(torch.from_numpy(tv), non_blocking=True)
        params = torch.from_numpy(pv).to(dev, non_blocking=True)
        out = buf.run_rows()
        ops.sched_step_rows(out, buf.lat, True, self.guidance, eng.scheduler.pred_type, params)
        self.stats["steps"] += 1
        self.stats["rows"] += n
        fin = []
        for j, r in enumerate(rows):
            r.i += 1
            if r.i >= len(r.steps):
                fin.append(j)
        if fin:
            with prof.range_("vae_decode"):
                for c0 in range(0, len(fin), self.VAE_MAX_BATCH):   # sizes warmed up by warmup()
                    part = fin[c0:c0 + self.VAE_MAX_BATCH]
                    img = eng.vae(buf.lat[part[0]:part[0] + 1] if len(part) == 1
                                  else buf.lat[torch.tensor(part, device=dev)])
                    u8 = AutoencoderKLDecoder.to_uint8(img).cpu()
                    now = time.perf_counter()
                    for k, j in enumerate(part):
                        rows[j].image, rows[j].done, rows[j].finish_time = u8[k], True, now
        self.active = rows
        return [rows[j] for j in fin]

    def _regroup(self, keep: List[DiffusionRequest], new: List[DiffusionRequest]):
        """Gather the kept requests' state rows and the new requests' fresh state into the bucket of the new
        row count (rows: kept requests in their previous order, then the new ones)."""
        eng, dev = self.eng, self.eng.device
        old, old_rows = self.buf, self.active
        n = len(keep) + len(new)
        Bc = self.bucket(n)
        if new:
            with prof.range_("text_encode"):
                ctx = eng.encode_prompts([r.prompt for r in new], [r.negative for r in new])
                kv_new = eng.unet.context_kv(ctx)      # per layer [2k, 77, C]: uncond k rows, then cond k rows
            if self._kv_shapes1 is None:
                self._kv_shapes1 = [t.shape[1:] for t in kv_new]
            lats = []
            for r in new:
                g = torch.Generator(device=dev)
                g.manual_seed(r.seed)
                lats.append(torch.randn(1, self.h, self.w, eng.cfg.unet.in_channels, generator=g, device=dev,
                                        dtype=torch.float32).mul_(eng.scheduler.init_noise_sigma).to(torch.bfloat16))
            lat_new = torch.cat(lats, 0)
        buf = self._buffers(Bc, [(2 * Bc,) + tuple(s) for s in self._kv_shapes1])
        k_old = len(keep)
        if k_old:
            pos = {id(r): i for i, r in enumerate(old_rows)}
            idx = torch.tensor([pos[id(r)] for r in keep], device=dev)
            ob = old.lat.shape[0]
            lat_keep = old.lat.index_select(0, idx)
            kv_keep = [(t.index_select(0, idx), t.index_select(0, idx + ob)) for t in old.kv]
        k = len(new)
        # every gathered piece is materialised before the (possibly same) destination buffers are written
        lat_parts = ([lat_keep] if k_old else []) + ([lat_new] if k else [])
        buf.lat[:n].copy_(torch.cat(lat_parts, 0) if len(lat_parts) > 1 else lat_parts[0])
        for l, dst in enumerate(buf.kv):
            unc = ([kv_keep[l][0]] if k_old else []) + ([kv_new[l][:k]] if k else [])
            cond = ([kv_keep[l][1]] if k_old else []) + ([kv_new[l][k:]] if k else [])
            dst[:n].copy_(torch.cat(unc, 0) if len(unc) > 1 else unc[0])
            dst[Bc:Bc + n].copy_(torch.cat(cond, 0) if len(cond) > 1 else cond[0])
        self.buf = buf


class _Rows:
    """Eager stand-in for :class:`_UNetGraph` (CPU / graphs off): same static state buffers, direct forward."""

    def __init__(self, unet, B, h, w, kv_shapes, device):
        self.unet = unet
        self.lat = torch.zeros(B, h, w, unet.cfg.in_channels, dtype=torch.bfloat16, device=device)
        self.t = torch.zeros(2 * B, dtype=torch.float32, device=device)
        self.kv = [torch.zeros(s, dtype=torch.bfloat16, device=device) for s in kv_shapes]

    def run_rows(self):
        return self.unet(torch.cat([self.lat, self.lat], 0), self.t, self.kv)


def to_pil(img_u8: torch.Tensor):
    from PIL import Image
    return Image.fromarray(np.ascontiguousarray(img_u8.numpy()))
