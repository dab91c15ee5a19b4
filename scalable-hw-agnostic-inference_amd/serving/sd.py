"""Stable Diffusion 2.1 server -- API-compatible with app/run-sd.py / app/run-sd2.py.

Routes (same paths, request and response JSON):
  GET  /                               -> {"message": "This is<model> pod <pod> ..."}
  GET  /load/{n_runs}/infer/{n_inf}    -> {"message": "benchmark report:RESULT FOR stable_diffusion_512 on <pod>: Latency P0=..."}
  POST /genimage {"prompt": str}       -> {"prompt", "response": base64 PNG, "latency": str(seconds)}
  GET  /health, /readiness, /metrics, /serve
Per-request metrics <APP>-counter / <NODEPOOL> / <APP>-latency as in run-sd.py:166-173.

Concurrent /genimage requests with the same step count are batched into one
CFG-batched UNet pass (``EngineWorker`` dynamic batching); the reference runs
one pipeline call per request on a shared, unsynchronised pipeline.
"""
from __future__ import annotations

import os
import time
from typing import Optional

from .common import METRICS, EngineWorker, ServerEnv, base_app, benchmark, mount_ui, png_b64, run

LOAD_PROMPT = "a photo of an astronaut riding a horse on mars"
WARMUP_PROMPT = "portrait photo of a old warrior chief"


def build_engine(env: ServerEnv):
    from ..engines.diffusion import SDConfig, StableDiffusionEngine
    cfg = SDConfig.tiny() if env.config == "tiny" else SDConfig.sd21(
        prediction_type="epsilon" if "base" in env.model_id else "v_prediction", height=env.height, width=env.width)
    return StableDiffusionEngine(cfg, device=env.torch_device, model_path=env.model_path)


def create_app(engine=None, env: Optional[ServerEnv] = None, max_batch: int = 8, title_suffix: str = ""):
    env = env or ServerEnv.from_env(app="sd21", num_inference_steps=50)
    engine = engine or build_engine(env)

    def batch_fn(steps, arg_lists):
        prompts = [a[0] for a in arg_lists]
        imgs = engine.generate(prompts, steps)
        return [imgs[i] for i in range(len(prompts))]

    worker = EngineWorker("sd-engine", batch_fn=batch_fn, max_batch=max_batch, max_wait_ms=10.0)

    def text2img(prompt: str, steps: Optional[int] = None):
        t0 = time.time()
        img = worker.submit_batched(int(steps or env.num_inference_steps), prompt).result()
        return img, str(time.time() - t0)

    # import-time warm-up, as the reference does (run-sd.py:144-146); it also captures the UNet-step HIP graph
    # of every batch size the dynamic batcher can form, so no request pays a capture later
    # (SHAI_WARMUP_ALL_BATCHES=0: batch size 1 only)
    def warm():
        engine.generate([WARMUP_PROMPT], min(env.num_inference_steps, 2))
        if os.environ.get("SHAI_WARMUP_ALL_BATCHES", "1") != "0":
            for b in range(2, max_batch + 1):
                engine.generate([WARMUP_PROMPT] * b, 1)
    worker.call(warm)

    app = base_app(env, f"{env.model_id} SD2.1{title_suffix}", spaced=False)
    app.state.engine, app.state.worker = engine, worker

    @app.get("/")
    def read_main():
        return {"message": "This is" + env.model_id + " pod " + env.pod_name + " in AWS EC2 " + env.device +
                " instance; try /load/{n_runs}/infer/{n_inf}; /genimage http post with user prompt "}

    @app.get("/load/{n_runs}/infer/{n_inf}")
    def load(n_runs: int, n_inf: int):
        t0 = time.time()
        report = benchmark(n_runs, "stable_diffusion_512",
                           lambda: worker.submit_batched(n_inf, LOAD_PROMPT).result(), env.pod_name)
        METRICS.request_done(env, time.time() - t0)
        return {"message": "benchmark report:" + report}

    @app.post("/genimage")
    def generate_image_post(request: dict):
        prompt = request.get("prompt")
        img, latency = text2img(prompt)
        METRICS.request_done(env, float(latency))
        return {"prompt": prompt, "response": png_b64(img), "latency": latency}

    mount_ui(app, f"{env.model_id} on MI355X; pod {env.pod_name}", "/genimage", "{prompt: p}", output="image")
    return app


def main():
    run(create_app())


if __name__ == "__main__":
    main()
