#!/usr/bin/env python3
"""Headline benchmark (driver contract).

Default workload: Stable Diffusion 2.1 512x512 txt2img, 50 DDIM steps, CFG 7.5,
bf16, random-init weights of the full SD2.1 architecture (UNet 865M, OpenCLIP-H
text encoder, VAE decoder), synthetic prompts.  One "step" = one batched
txt2img request of ``--batch`` images per GPU (text encode + 50 UNet steps +
VAE decode) -- nothing is skipped inside the timed region.  N GPUs run N
data-parallel replicas (one process per GPU, torch.distributed over RCCL for
the barrier / max-reduction), so per-GPU work is fixed: weak scaling.

``--workload flux``: Flux.1-dev 512x512 (10 steps by default) images/s + p50 latency.

``--workload mistral``: Mistral-7B bf16 decode throughput (tokens/s) through the
native LLM engine at TP = N (see shai_amd.engines.llm).

``--workload vit``: ViT-base/16 224x224 classification images/s at batch 32 per GPU.

``--tp T`` (mistral / flux): tensor-parallel degree of one replica; the N GPUs run N / T replicas
(data parallel x tensor parallel).  Defaults: mistral T = N (one engine over all GPUs, strong scaling),
flux T = 1 (one replica per GPU).  ``--workload flux --tp 8`` is the reference's Flux TP8 latency setup
(cova/README.md:98).

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--tp T]
        python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
``python bench.py --gpus N`` with N > 1 outside a launcher re-runs itself under torch.distributed.run with N
ranks (a child process, started before this process touches the GPU).  Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# Reference's best published per-accelerator SD2.1 rate: trn1.2xlarge breaking point
# 130 requests / CloudWatch period (= per minute), one 512^2 image per
# request at an unpublished (smaller) step count; we compare 50-step images/s to it.
REF_SD21_IMG_PER_S = 130.0 / 60.0


def _relaunch(n):
    """``--gpus N`` without a launcher: run N ranks under torch.distributed.run (127.0.0.1 rendezvous) as a
    child process and exit with its status.  Nothing here has touched the GPU yet."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    sys.exit(subprocess.call(cmd))


# --cpu-dry-run: the multi-process plumbing (launcher, rendezvous, barriers, max over ranks, JSON line) on a
# tiny config over gloo on the CPU -- for tests; NOT a measurement.
DEVICE = "cuda"


def _sync():
    import torch
    if DEVICE == "cuda":
        torch.cuda.synchronize()


def _dist_init(n):
    import torch
    import torch.distributed as dist
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != n:
        raise SystemExit(f"bench.py --gpus {n} but WORLD_SIZE={world}: launch {n} ranks (or run without a launcher)")
    if DEVICE == "cpu":
        if world > 1 and not dist.is_initialized():
            dist.init_process_group("gloo")
        return rank, world, local
    if world > 1:
        torch.cuda.set_device(local)
        if not dist.is_initialized():
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    return rank, world, local


def _groups(args, world):
    """(tp, replicas, replica index of this rank): consecutive ranks form one TP group."""
    tp = args.tp or 1
    if world % tp:
        raise SystemExit(f"--tp {tp} does not divide --gpus {world}")
    rank = int(os.environ.get("RANK", "0"))
    return tp, world // tp, rank // tp


def _barrier(world):
    import torch.distributed as dist
    _sync()
    if world > 1:
        dist.barrier()
        _sync()


def _max_over_ranks(x, world):
    import torch
    import torch.distributed as dist
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=DEVICE)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def bench_sd21(args, rank, world):
    import torch
    from shai_amd.engines.diffusion import SDConfig, StableDiffusionEngine

    cfg = SDConfig.tiny() if DEVICE == "cpu" else SDConfig.sd21(height=args.height, width=args.width)
    eng = StableDiffusionEngine(cfg, device=DEVICE, seed=rank, use_graphs=not args.no_graphs)
    prompts = [f"a photo of an astronaut riding a horse on mars, variant {rank}-{i}" for i in range(args.batch)]
    for i in range(args.warmup):
        eng.generate(prompts, args.inference_steps, seed=1000 + i, output="tensor")
    # p50 single-image latency (reference's request latency semantics), outside the timed region
    lat = []
    for i in range(args.latency_runs):
        _sync()
        t0 = time.perf_counter()
        eng.generate(prompts[:1], args.inference_steps, seed=2000 + i)
        _sync()
        lat.append(time.perf_counter() - t0)
    _barrier(world)
    t0 = time.perf_counter()
    per = []
    for i in range(args.steps):
        s0 = time.perf_counter()
        img = eng.generate(prompts, args.inference_steps, seed=3000 + i, output="tensor")
        _sync()
        per.append(time.perf_counter() - s0)
    _barrier(world)
    elapsed = _max_over_ranks(time.perf_counter() - t0, world)
    ok = bool(torch.isfinite(img.float()).all().item())
    images = args.batch * args.steps * world
    value = images / elapsed
    res = {
        "metric": "SD2.1 512x512 images/sec (50 DDIM steps, CFG 7.5)" if args.inference_steps == 50 and
        args.height == 512 else f"SD2.1 {args.height}x{args.width} images/sec ({args.inference_steps} steps)",
        "value": round(value, 4),
        "unit": "images/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1000 * elapsed / args.steps, 2),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(value / REF_SD21_IMG_PER_S, 3),
        "dtype": "bf16",
        "data": "synthetic prompts, random-init weights (full SD2.1 architecture)",
        "config": {"model": "stabilityai/stable-diffusion-2-1 (UNet2DCondition 865M + OpenCLIP-H text + VAE)",
                   "global_batch": args.batch * world, "per_gpu_batch": args.batch, "seq_len": 77,
                   "resolution": f"{args.height}x{args.width}", "inference_steps": args.inference_steps,
                   "guidance_scale": 7.5, "scheduler": "DDIM", "parallelism": f"dp{world}",
                   "hip_graphs": not args.no_graphs},
        "p50_latency_ms_bs1": round(1000 * statistics.median(lat), 1) if lat else None,
        "p50_batch_latency_ms": round(1000 * statistics.median(per), 1),
        "baseline_note": "vs_baseline = images/s / (130/60): reference trn1 SD2.1 breaking-point 130 req/min/pod "
                         "(README.md:193), unpublished step count (<=50)",
        "outputs_finite": ok,
    }
    return res


REF_FLUX_512_10STEP_S = 5.61   # cova/README.md:98 (Neuron TP8 Flux service, 512x512, 10 steps, end-to-end)


def bench_flux(args, rank, world):
    """Flux.1-dev txt2img (CLIP-L + T5-XXL 512 tokens + 12B MMDiT + 16-ch VAE).  ``--tp T``: each replica is
    a TP group of T GPUs (MMDiT + T5 sharded, collectives over RCCL / the xGMI P2P kernel); default one
    replica per GPU."""
    import torch
    from shai_amd.engines.flux import FluxEngine, FluxPipelineConfig
    from shai_amd.parallel.state import init_distributed
    tp, replicas, rep = _groups(args, world)
    init_distributed(tp_size=tp)
    steps_inf = args.inference_steps if args.inference_steps != 50 else 10
    eng = FluxEngine(FluxPipelineConfig.dev(args.height, args.width, 512), device="cuda", seed=0,
                     use_graphs=not args.no_graphs)
    prompts = [f"A cat holding a sign that says hello world, variant {rep}-{i}" for i in range(args.batch)]
    for i in range(args.warmup):
        eng.generate(prompts, steps_inf, seed=10 + i, output="tensor")
    lat = []
    for i in range(args.latency_runs):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.generate(prompts[:1], steps_inf, seed=20 + i)
        torch.cuda.synchronize()
        lat.append(time.perf_counter() - t0)
    _barrier(world)
    t0 = time.perf_counter()
    for i in range(args.steps):
        img = eng.generate(prompts, steps_inf, seed=30 + i, output="tensor")
    torch.cuda.synchronize()
    _barrier(world)
    elapsed = _max_over_ranks(time.perf_counter() - t0, world)
    value = args.batch * args.steps * replicas / elapsed
    p50 = statistics.median(lat) if lat else None
    return {
        "metric": f"Flux.1-dev {args.height}x{args.width} images/sec ({steps_inf} steps)",
        "value": round(value, 4), "unit": "images/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(1000 * elapsed / args.steps, 2), "higher_is_better": True,
        "scaling": "weak" if tp == 1 else "strong",
        "vs_baseline": round(REF_FLUX_512_10STEP_S / p50, 3) if (p50 and steps_inf == 10 and args.height == 512)
        else None,
        "dtype": "bf16", "data": "synthetic prompts, random-init weights (full Flux.1-dev architecture)",
        "config": {"model": "black-forest-labs/FLUX.1-dev (MMDiT 11.9B + T5-XXL + CLIP-L + VAE)",
                   "global_batch": args.batch * replicas, "per_replica_batch": args.batch, "seq_len": 512,
                   "resolution": f"{args.height}x{args.width}", "inference_steps": steps_inf,
                   "guidance_scale": 3.5, "parallelism": f"dp{replicas}" + (f"xtp{tp}" if tp > 1 else ""),
                   "hip_graphs": not args.no_graphs},
        "p50_latency_ms_bs1": round(1000 * p50, 1) if p50 else None,
        "baseline_note": "vs_baseline = 5.61 s (reference Flux 512^2 10-step end-to-end on Neuron TP8, "
                         "cova/README.md:98) / our p50 single-image latency",
        "outputs_finite": bool(torch.isfinite(img.float()).all().item()),
    }


REF_MLLAMA_CAPTION_S = 5.70   # cova/README.md:98 (Llama-3.2-11B-Vision caption, trn1, vLLM TP32)


def bench_mllama(args, rank, world):
    """Llama-3.2-11B-Vision image captioning (the cova caption stage): one 4-tile image + instruct prompt per
    request, ``gen_len`` sampled tokens; captions/s over ``batch`` concurrent requests + p50 bs1 latency."""
    import numpy as np
    import torch
    from shai_amd.engines.llm import LLMEngine, SamplingParams
    from shai_amd.models.mllama import MllamaConfig, preprocess_image
    from shai_amd.parallel.state import init_distributed
    init_distributed(tp_size=world)
    mc = MllamaConfig.llama32_11b_vision()
    B, G = max(1, args.batch), args.gen_len
    eng = LLMEngine(mc, device=f"cuda:{torch.cuda.current_device()}", max_num_seqs=B, max_model_len=64 + G + 64,
                    enable_prefix_caching=False)
    rng = np.random.default_rng(rank)
    img = (rng.random((1024, 1024, 3)) * 255).astype(np.uint8)            # -> 2x2 tiles of 560^2
    pre = preprocess_image(img, mc.vision, eng.device)
    t = mc.text
    prompt = [t.bos_token_id, mc.image_token_index] + rng.integers(1000, 100000, 24).tolist()
    params = SamplingParams(temperature=0.7, top_k=50, top_p=0.9, max_tokens=G, ignore_eos=True)
    for _ in range(max(1, args.warmup)):
        for _ in range(B):
            eng.add_request(prompt, params, image=pre)
        while eng.has_work():
            eng.step()
    lat = []
    for _ in range(args.latency_runs):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        s = eng.add_request(prompt, params, image=pre)
        while not s.finished:
            eng.step()
        torch.cuda.synchronize()
        lat.append(time.perf_counter() - t0)
    _barrier(world)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        for _ in range(B):
            eng.add_request(prompt, params, image=pre)
        while eng.has_work():
            eng.step()
    torch.cuda.synchronize()
    _barrier(world)
    el = _max_over_ranks(time.perf_counter() - t0, world)
    p50 = statistics.median(lat) if lat else None
    n = B * args.steps
    return {
        "metric": "Llama-3.2-11B-Vision captions/sec (4-tile image, %d tokens)" % G,
        "value": round(n / el, 4), "unit": "captions/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(1000 * el / args.steps, 2), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": round(REF_MLLAMA_CAPTION_S / p50, 3) if p50 else None,
        "dtype": "bf16", "data": "synthetic image + prompt, random-init weights (full Llama-3.2-11B-Vision)",
        "config": {"model": "meta-llama/Llama-3.2-11B-Vision-Instruct (architecture)", "global_batch": B,
                   "seq_len": len(prompt) + G, "gen_len": G, "image_tiles": pre["num_tiles"],
                   "parallelism": f"tp{world}"},
        "p50_latency_ms_bs1": round(1000 * p50, 1) if p50 else None,
        "tokens_per_s": round(n * G / el, 1),
        "baseline_note": "vs_baseline = 5.70 s (reference mllama caption latency, cova/README.md:98) / our p50 "
                         "single-request latency",
    }


def bench_vit(args, rank, world):
    """ViT-base/16 224x224 image classification (run-vit.py; BASELINE.json config 2: batch 32 per GPU).
    One step = one batch: uint8 images -> normalise -> 12-layer encoder -> classifier -> argmax labels on
    the host (a HIP graph per batch size).  The reference publishes no ViT number: vs_baseline is null."""
    import torch
    from shai_amd.engines.encoders import ImageClassifierEngine
    from shai_amd.models.vit import ViTConfig

    eng = ImageClassifierEngine(ViTConfig.vit_base(), device="cuda", seed=rank, use_graphs=not args.no_graphs)
    g = torch.Generator(device="cuda")
    g.manual_seed(rank)
    imgs = torch.randint(0, 256, (args.batch, 224, 224, 3), device="cuda", dtype=torch.uint8, generator=g)
    for _ in range(max(1, args.warmup)):
        eng.logits_u8(imgs).argmax(-1).cpu()
    lat = []
    for _ in range(args.latency_runs):  # single-image request latency (reference semantics), untimed
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.logits_u8(imgs[:1]).argmax(-1).cpu()
        lat.append(time.perf_counter() - t0)
    _barrier(world)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        labels = eng.logits_u8(imgs).argmax(-1).cpu()
    _barrier(world)
    elapsed = _max_over_ranks(time.perf_counter() - t0, world)
    value = args.batch * args.steps * world / elapsed
    return {
        "metric": "ViT-base/16 224x224 images/sec (image classification)", "value": round(value, 2),
        "unit": "images/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(1000 * elapsed / args.steps, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "bf16", "data": "synthetic uint8 images, random-init weights",
        "config": {"model": "google/vit-base-patch16-224 (architecture)", "global_batch": args.batch * world,
                   "per_gpu_batch": args.batch, "seq_len": 197, "parallelism": f"dp{world}",
                   "hip_graphs": not args.no_graphs},
        "p50_latency_ms_bs1": round(1000 * statistics.median(lat), 3) if lat else None,
        "labels_in_range": bool(((labels >= 0) & (labels < 1000)).all().item()),
    }


REF_T5_CAPTION_S = 0.20  # reference T5-v1.1-large caption embedding latency, inf2 (cova/README.md:98)


def bench_t5(args, rank, world):
    """T5-v1.1-large mean-pooled embeddings (t5_model_api.py / the cova chain).  One step = one batch of
    ``--batch`` captions padded to ``--prompt-len`` tokens (the server's ``max_new_tokens``); the reference's
    single-request caption / prompt embedding latencies (0.20 s / 0.09 s, inf2) are matched by the p50 of
    single requests at the same length.  Eager encoder (no graph), tokenizer on the host included."""
    import numpy as np
    import torch
    from shai_amd.engines.encoders import TextEmbeddingEngine
    from shai_amd.models.t5 import T5Config

    eng = TextEmbeddingEngine(T5Config.v1_1_large(), device="cuda", seed=rank)
    L = args.prompt_len
    caption = ("a photograph of an astronaut riding a horse on the surface of mars, dramatic lighting, "
               "red dust, highly detailed")
    texts = [caption] * args.batch
    for _ in range(max(1, args.warmup)):
        eng.embed(texts, L)
        eng.embed(texts[:1], L)
    lat = []
    for _ in range(max(args.latency_runs, 5)):  # single-request latency (reference semantics), untimed
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e = eng.embed(texts[:1], L)
        lat.append(time.perf_counter() - t0)
    _barrier(world)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        e = eng.embed(texts, L)
    _barrier(world)
    elapsed = _max_over_ranks(time.perf_counter() - t0, world)
    p50 = statistics.median(lat)
    return {
        "metric": "T5-v1.1-large embeddings/sec (mean-pooled, %d tokens)" % L, "value": round(args.batch * args.steps * world / elapsed, 2),
        "unit": "embeddings/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(1000 * elapsed / args.steps, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": round(REF_T5_CAPTION_S / p50, 3), "dtype": "bf16",
        "data": "synthetic caption, random-init weights (full T5-v1.1-large encoder)",
        "config": {"model": "google/t5-v1_1-large (encoder architecture)", "global_batch": args.batch * world,
                   "per_gpu_batch": args.batch, "seq_len": L, "parallelism": f"dp{world}"},
        "p50_latency_ms_bs1": round(1000 * p50, 2),
        "embedding_dim": int(e.shape[-1]), "outputs_finite": bool(np.isfinite(e).all()),
        "baseline_note": "vs_baseline = 0.20 s (reference T5 caption embedding latency, inf2, cova/README.md:98) / our "
                         "p50 single-request latency",
    }


def bench_mistral(args, rank, world):
    import torch
    from shai_amd.engines.llm import bench_decode_throughput
    return bench_decode_throughput(args, rank, world)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default="sd21", choices=["sd21", "mistral", "flux", "mllama", "vit", "t5"])
    ap.add_argument("--batch", type=int, default=None,
                    help="per-GPU batch: images per step (sd21: 32, flux: 1) / concurrent sequences (mistral: 64, "
                         "mllama: 8)")
    ap.add_argument("--inference-steps", type=int, default=50)
    ap.add_argument("--height", type=int, default=512)
    ap.add_argument("--width", type=int, default=512)
    ap.add_argument("--quantization", default=None, choices=[None, "fp8"],
                    help="mistral: fp8 e4m3 weight-only quantisation (NOT the bf16 headline config)")
    ap.add_argument("--latency-runs", type=int, default=3)
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--prompt-len", type=int, default=128)
    ap.add_argument("--gen-len", type=int, default=128)
    ap.add_argument("--llm-model", default="mistral_7b", choices=["mistral_7b", "llama3_8b", "deepseek_r1_distill_70b"],
                    help="--workload mistral: which Llama-architecture model (BASELINE config 4 is mistral_7b)")
    ap.add_argument("--cpu-dry-run", action="store_true",
                    help="tests only: tiny SD2.1 config on the CPU over gloo (launcher / rendezvous / JSON plumbing)")
    ap.add_argument("--tp", type=int, default=None,
                    help="tensor-parallel degree per replica (mistral default: --gpus; flux default: 1)")
    args = ap.parse_args()
    global DEVICE
    if args.cpu_dry_run:
        DEVICE = "cpu"
        args.no_graphs = True
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        _relaunch(args.gpus)
    if args.tp is None:
        args.tp = args.gpus if args.workload in ("mistral", "mllama") else 1
    if args.batch is None:  # dynamic-batching caps a serving replica would use for each workload
        args.batch = {"sd21": 32, "mistral": 64, "flux": 1, "mllama": 8, "vit": 32, "t5": 32}[args.workload]
    import torch
    rank, world, local = _dist_init(args.gpus)
    with torch.inference_mode():
        fn = {"sd21": bench_sd21, "mistral": bench_mistral, "flux": bench_flux,
              "mllama": bench_mllama, "vit": bench_vit, "t5": bench_t5}[args.workload]
        res = fn(args, rank, world)
    if DEVICE == "cpu":
        res["data"] = "CPU DRY RUN (tiny config, gloo): plumbing check, not a measurement"
    if rank == 0:
        print(json.dumps(res), flush=True)
        save = os.environ.get("SHAI_GEMM_TUNE_SAVE")
        if save:
            import shai_amd.native as native
            native.save_gemm_tuning(save)
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
