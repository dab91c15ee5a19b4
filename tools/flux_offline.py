#!/usr/bin/env python3
"""Standalone Flux.1-dev text-to-image run (no server): load, generate one image, save a PNG.

Counterpart of the reference's offline Neuron script app/src/inference.py:168-250 (same CLI:
-p/--prompt, -hh/--height, -w/--width, -m/--max_sequence_length, -n/--num_inference_steps; guidance 3.5,
output ``flux-dev.png``).  There is no compile step: the native engine captures one HIP graph per
(batch, text length, latent grid) bucket at the first call.  ``--tp N`` under torchrun shards the
MMDiT and T5-XXL across N GPUs (RCCL over xGMI); rank 0 writes the image.

    python tools/flux_offline.py -p "A cat holding a sign that says hello world" -hh 1024 -w 1024 -n 50
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 tools/flux_offline.py --tp 8
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("-p", "--prompt", default="A cat holding a sign that says hello world")
    ap.add_argument("-hh", "--height", type=int, default=1024)
    ap.add_argument("-w", "--width", type=int, default=1024)
    ap.add_argument("-m", "--max_sequence_length", type=int, default=512)
    ap.add_argument("-n", "--num_inference_steps", type=int, default=50)
    ap.add_argument("--model-path", default=os.environ.get("MODEL_PATH"), help="local diffusers checkpoint dir")
    ap.add_argument("--config", default="dev", choices=["dev", "schnell", "tiny"])
    ap.add_argument("--tp", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--out", default="flux-dev.png")
    ap.add_argument("--device", default=None)
    a = ap.parse_args(argv)

    import torch
    from shai_amd.engines.flux import FluxEngine, FluxPipelineConfig
    from shai_amd.engines.diffusion import to_pil
    from shai_amd.parallel.state import init_distributed

    st = init_distributed(tp_size=a.tp) if a.tp > 1 else None
    dev = a.device or (str(st.device) if st is not None else ("cuda" if torch.cuda.is_available() else "cpu"))
    cfg = {"dev": FluxPipelineConfig.dev, "schnell": FluxPipelineConfig.schnell,
           "tiny": lambda *x: FluxPipelineConfig.tiny()}[a.config](a.height, a.width, a.max_sequence_length)
    eng = FluxEngine(cfg, device=dev, model_path=a.model_path, seed=a.seed)
    with torch.inference_mode():
        t0 = time.perf_counter()
        img = eng.generate([a.prompt], a.num_inference_steps, height=cfg.height, width=cfg.width, seed=a.seed,
                           max_sequence_length=min(a.max_sequence_length, cfg.max_sequence_length))
        dt = time.perf_counter() - t0
    if st is None or st.rank == 0:
        to_pil(img[0]).save(a.out)
        print(f"wrote {a.out} ({img.shape[2]}x{img.shape[1]}) in {dt:.2f}s; weights: {eng.weights}", flush=True)
    return img


if __name__ == "__main__":
    main()
