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
    """HIP-graph-captured UNet forward for one (batch, latent HxW) bucket."""

    def __init__(self, unet: UNet2DConditionModel, B: int, h: int, w: int, ctx_len: int, ctx_shapes, device):
        self.unet = unet
        self.lat = torch.zeros(B, h, w, unet.cfg.in_channels, dtype=torch.bfloat16, device=device)
        self.t = torch.zeros(1, dtype=torch.float32, device=device)
        self.kv = [torch.zeros(s, dtype=torch.bfloat16, device=device) for s in ctx_shapes]
        self.graph = new_graph(device)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                self._fwd()
        torch.cuda.current_stream().wait_stream(s)
        with torch.cuda.graph(self.graph):
            self.out = self._fwd()

    def _fwd(self):
        x = torch.cat([self.lat, self.lat], 0)
        return self.unet(x, self.t, self.kv)

    def run(self, t: float) -> torch.Tensor:
        self.t.fill_(t)
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


def to_pil(img_u8: torch.Tensor):
    from PIL import Image
    return Image.fromarray(np.ascontiguousarray(img_u8.numpy()))
