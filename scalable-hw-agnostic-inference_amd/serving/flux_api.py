"""Flux.1 servers -- API-compatible with app/flux_model_api.py (JSON) and
app/run-flux.py (Gradio UI).

flux_model_api.py-compatible routes (``create_app``):
  POST /generate {"prompt": str, "num_inference_steps": int}
       -> {"image": base64 PNG 128x128 thumbnail (LANCZOS), "execution_time": float}
       errors -> 500 {"detail": "Image serialization failed: <err>"} (the reference's
       handler references an undefined name there, flux_model_api.py:362)
  GET  /health, /readiness  -> "<pod> is healthy" / "<pod> is ready"
run-flux.py-compatible routes (``create_gradio_app``):
  POST /text2img {"prompt", "num_inference_steps"} -> {"image": full-size base64 PNG, "execution_time": str}
  GET  /serve (UI), /health, /readiness -> "<pod>is healthy" (no space, run-flux.py:269-275)
Env: MODEL_ID, HEIGHT, WIDTH, MAX_SEQ_LEN, GUIDANCE_SCALE, APP, POD_NAME, NODEPOOL
(flux_model_api.py:27-37).  Warm-up at start-up as the reference (benchmark(10, ...),
flux_model_api.py:322-328; here 1 run by default, FLUX_WARMUP_RUNS overrides).

Concurrent requests with the same step count are batched into one transformer
pass per step (EngineWorker dynamic batching).

Tensor parallelism (the reference's transformer TP8, flux_model_api.py:128-140, and T5
TP8, :312-314): ``TENSOR_PARALLEL_SIZE=N`` runs the worker as N ranks (one GPU each,
torch.distributed.run); every rank holds its shard of the MMDiT / T5 and rank 0 broadcasts
each batched ``generate`` call (prompts, steps, seed) to the others (serving/tp.py).
"""
import os
import secrets
import time
from typing import Optional

from pydantic import BaseModel

from .common import METRICS, EngineWorker, ServerEnv, base_app, benchmark, mount_ui, png_b64

WARMUP_PROMPT = "A cat holding a sign that says hello world"


class GenerateImageRequest(BaseModel):
    prompt: str
    num_inference_steps: int = 28


class GenerateImageResponse(BaseModel):
    image: str
    execution_time: float


def build_engine(env: ServerEnv):
    from ..engines.flux import FluxEngine, FluxPipelineConfig
    if env.config == "tiny":
        cfg = FluxPipelineConfig.tiny()
    elif "schnell" in env.model_id.lower():
        cfg = FluxPipelineConfig.schnell(env.height, env.width, env.max_seq_len)
    else:
        cfg = FluxPipelineConfig.dev(env.height, env.width, env.max_seq_len)
        cfg.guidance_scale = env.guidance_scale
    return FluxEngine(cfg, device=env.torch_device, model_path=env.model_path)


def _worker(engine, env: ServerEnv, max_batch: int):
    def batch_fn(steps, arg_lists):
        # explicit seed: at TP > 1 every rank must draw the same initial noise (SHAI_SEED pins it)
        seed = int(os.environ["SHAI_SEED"]) if os.environ.get("SHAI_SEED") else secrets.randbits(31)
        imgs = engine.generate([a[0] for a in arg_lists], steps, seed=seed)
        return [imgs[i] for i in range(len(arg_lists))]

    w = EngineWorker("flux-engine", batch_fn=batch_fn, max_batch=max_batch, max_wait_ms=10.0)
    runs = int(os.environ.get("FLUX_WARMUP_RUNS", "1"))
    test_name = (f"flux1-dev-{runs}runs with dim {env.height}x{env.width} on {env.nodepool};"
                 f"num_inference_steps:{min(env.num_inference_steps, 10)}")
    w.call(lambda: print(benchmark(runs, test_name, lambda: engine.generate([WARMUP_PROMPT],
                                                                           min(env.num_inference_steps, 10),
                                                                           seed=0),
                                   env.pod_name, warmup=True)))
    return w


def _env():
    return ServerEnv.from_env(app="flux", model_id="black-forest-labs/FLUX.1-dev", num_inference_steps=28)


def _engine(engine, env, tpc):
    engine = engine or build_engine(env)
    return tpc.wrap(engine, ("generate",)) if tpc is not None else engine


def create_app(engine=None, env: Optional[ServerEnv] = None, max_batch: int = 4, tpc=None):
    env = env or _env()
    engine = _engine(engine, env, tpc)
    worker = _worker(engine, env, max_batch)
    app = base_app(env, f"{env.model_id} Flux API", spaced=True)
    app.state.engine, app.state.worker = engine, worker

    @app.post("/generate", response_model=GenerateImageResponse)
    def generate_image(request: GenerateImageRequest):
        from fastapi import HTTPException
        t0 = time.time()
        try:
            img = worker.submit_batched(int(request.num_inference_steps), request.prompt).result()
            image_b64 = png_b64(img, thumbnail=128)
            total = time.time() - t0
            METRICS.request_done(env, total)
            return GenerateImageResponse(image=image_b64, execution_time=total)
        except Exception as e:  # noqa: BLE001 -- reference contract: every failure is a 500 with this prefix
            raise HTTPException(status_code=500, detail=f"Image serialization failed: {e}")

    mount_ui(app, f"{env.model_id} on MI355X; pod {env.pod_name}", "/generate",
             "{prompt: p, num_inference_steps: 28}", output="image")
    return app


def create_gradio_app(engine=None, env: Optional[ServerEnv] = None, max_batch: int = 4, tpc=None):
    """run-flux.py equivalent: UI at /serve driving text2img(prompt, steps) -> (image, execution time)."""
    env = env or _env()
    engine = _engine(engine, env, tpc)
    worker = _worker(engine, env, max_batch)
    app = base_app(env, f"{env.model_id} in MI355X {env.device} instance; pod name {env.pod_name}", spaced=False)
    app.state.engine, app.state.worker = engine, worker

    @app.post("/text2img")
    def text2img(request: dict):
        t0 = time.time()
        steps = int(request.get("num_inference_steps") or env.num_inference_steps)
        img = worker.submit_batched(steps, request.get("prompt", "")).result()
        total = time.time() - t0
        METRICS.request_done(env, total)
        return {"image": png_b64(img), "execution_time": str(total)}

    mount_ui(app, f"{env.model_id} in MI355X {env.device} instance; pod name {env.pod_name}", "/text2img",
             "{prompt: p, num_inference_steps: 28}", output="image")
    return app


def main():
    from . import tp as tp_serving
    env = _env()
    make = create_gradio_app if os.environ.get("FLUX_UI", "") == "gradio" else create_app
    tp_serving.serve("shai_amd.serving.flux_api", tp_serving.env_tp_degree(), lambda: build_engine(env),
                     lambda tpc: make(env=env, tpc=tpc))


if __name__ == "__main__":
    main()
