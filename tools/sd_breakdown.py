"""Where one SD2.1 generate's time goes (GPU events): text encoder + context K/V, the 50 graph-replayed UNet steps,
the VAE decode -- at the bench batch (32) and at batch 1 (the p50 latency request).
    python tools/sd_breakdown.py [--batches 32,1] [--steps 50]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from shai_amd import ops  # noqa: E402
from shai_amd.engines.diffusion import SDConfig, StableDiffusionEngine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="32,1")
    ap.add_argument("--steps", type=int, default=50)
    a = ap.parse_args()
    eng = StableDiffusionEngine(SDConfig.sd21(), device="cuda", seed=0)
    for B in [int(x) for x in a.batches.split(",")]:
        prompts = [f"a photo of an astronaut riding a horse on mars, variant {i}" for i in range(B)]
        eng.generate(prompts, a.steps, seed=1, output="tensor")  # warm: graph capture, tuning
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        with torch.no_grad():
            t0 = time.perf_counter()
            ev[0].record()
            ctx = eng.encode_prompts(prompts)
            ctx_kv = eng.unet.context_kv(ctx)
            ev[1].record()
            h = w = 64
            lat = torch.randn(B, h, w, 4, device="cuda").to(torch.bfloat16)
            g = eng._graph_for(B, h, w, ctx_kv)
            for dst, src in zip(g.kv, ctx_kv):
                dst.copy_(src)
            g.lat.copy_(lat)
            for sp in eng.scheduler.steps(a.steps):
                out = g.run(sp.t)
                ops.sched_step(out, g.lat, True, 7.5, eng.scheduler.pred_type, sp.a_t, sp.a_prev)
            ev[2].record()
            eng.vae(g.lat)
            ev[3].record()
            torch.cuda.synchronize()
            wall = time.perf_counter() - t0
        te, un, va = (ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2]), ev[2].elapsed_time(ev[3]))
        print(f"B={B}: wall {wall * 1e3:.1f} ms | text+ctx_kv {te:.1f} ms | unet x{a.steps} {un:.1f} ms "
              f"({un / a.steps:.2f} ms/step) | vae {va:.1f} ms", flush=True)


if __name__ == "__main__":
    main()
