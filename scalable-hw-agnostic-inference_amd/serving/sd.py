"""Stable Diffusion 2.1 server -- API-compatible with app/run-sd.py / app/run-sd2.py.

Routes (same paths, request and response JSON):
  GET  /                               -> {"message": "This is<model> pod <pod> ..."}
  GET  /load/{n_runs}/infer/{n_inf}    -> {"message": "benchmark report:RESULT FOR stable_diffusion_512 on <pod>: Latency P0=..."}
  POST /genimage {"prompt": str}       -> {"prompt", "response": base64 PNG, "latency": str(seconds)}
  GET  /health, /readiness, /metrics, /serve
Per-request metrics <APP>-counter / <NODEPOOL> / <APP>-latency as in run-sd.py:166-173.

Step-level batching (default, ``SHAI_SD_STEP_BATCHING=1``): requests join the
running CFG-batched UNet batch at the next denoising-step boundary and leave it
when their own schedule ends (``engines.diffusion.StepBatcher``), so a request
never waits for another request's 50 steps; ``SHAI_SD_MAX_BATCH`` (default 32)
caps the rows.  ``SHAI_SD_STEP_BATCHING=0``: the older request-level batching
(concurrent requests with the same step count run as one batch,
``EngineWorker``).  The reference runs one pipeline call per request on a shared,
unsynchronised pipeline.
"""
from __future__ import annotations

import os
import queue
import threading
import time
from concurrent.futures import Future
from typing import Optional

from ..engines.diffusion import validate_request
from .common import METRICS, EngineWorker, ServerEnv, base_app, benchmark, mount_ui, png_b64, run

LOAD_PROMPT = "a photo of an astronaut riding a horse on mars"
WARMUP_PROMPT = "portrait photo of a old warrior chief"


def build_engine(env: ServerEnv):
    from ..engines.diffusion import SDConfig, StableDiffusionEngine
    cfg = SDConfig.tiny() if env.config == "tiny" else SDConfig.sd21(
        prediction_type="epsilon" if "base" in env.model_id else "v_prediction", height=env.height, width=env.width)
    return StableDiffusionEngine(cfg, device=env.torch_device, model_path=env.model_path)


class StepBatchingWorker:
    """The engine thread of step-level batching: drains the request queue into the StepBatcher before every
    denoising step, runs the step, resolves the finished requests' futures.  ``live`` reports progress per
    step to /health (a hung UNet step turns the replica unhealthy)."""

    def __init__(self, batcher):
        from ..utils.liveness import Liveness, register
        self.batcher = batcher
        self.q: "queue.Queue" = queue.Queue()
        self.live = register(Liveness())
        self._futs = {}
        self.t = threading.Thread(target=self._loop, name="sd-step-engine", daemon=True)
        self.t.start()

    def submit(self, prompt: str, steps: int, seed: Optional[int] = None) -> Future:
        validate_request(prompt, steps)
        f: Future = Future()
        self.live.work_pending()
        self.q.put((prompt, int(steps), seed, f))
        return f

    def call(self, fn, *args):
        """Run fn on the engine thread (warm-up); returns its result."""
        f: Future = Future()
        self.q.put((fn, args, None, f))
        return f.result()

    def _loop(self):
        import torch
        b = self.batcher
        while True:
            items = []
            try:
                block = not b.has_work()
                while True:
                    items.append(self.q.get(block=block))
                    block = False
            except queue.Empty:
                pass
            for a, steps, seed, f in items:
                if callable(a):   # engine-thread call
                    try:
                        with torch.inference_mode():
                            f.set_result(a(*steps))
                    except BaseException as e:  # noqa: BLE001
                        f.set_exception(e)
                    continue
                try:
                    self._futs[id(b.add(a, steps, seed))] = f
                except BaseException as e:  # noqa: BLE001 -- a bad request fails alone, before it joins the batch
                    f.set_exception(e)
            if not b.has_work():
                continue
            try:
                with torch.inference_mode():
                    done = b.step()
            except BaseException as e:  # noqa: BLE001 -- fail every request in the batch, reset it
                for f in self._futs.values():
                    if not f.done():
                        f.set_exception(e)
                self._futs.clear()
                b.waiting, b.active, b.buf = [], [], None
                continue
            for r in done:
                f = self._futs.pop(id(r), None)
                if f is not None:
                    f.set_result(r.image)
            self.live.progress(still_pending=b.has_work() or not self.q.empty())


def _check(prompt, steps) -> None:
    """Route-level validation: a malformed request is a 422 for its caller, never an engine-thread failure."""
    from fastapi import HTTPException
    try:
        validate_request(prompt, steps)
    except ValueError as e:
        raise HTTPException(status_code=422, detail=str(e)) from None


def create_app(engine=None, env: Optional[ServerEnv] = None, max_batch: Optional[int] = None, title_suffix: str = ""):
    env = env or ServerEnv.from_env(app="sd21", num_inference_steps=50)
    engine = engine or build_engine(env)
    step_batching = os.environ.get("SHAI_SD_STEP_BATCHING", "1") != "0"
    if max_batch is None:
        max_batch = int(os.environ.get("SHAI_SD_MAX_BATCH", "32" if step_batching else "8"))
    if step_batching:
        return _create_step_app(engine, env, max_batch, title_suffix)

    def batch_fn(steps, arg_lists):
        prompts = [a[0] for a in arg_lists]
        imgs = engine.generate(prompts, steps)
        return [imgs[i] for i in range(len(prompts))]

    worker = EngineWorker("sd-engine", batch_fn=batch_fn, max_batch=max_batch, max_wait_ms=10.0)

    def text2img(prompt: str, steps: Optional[int] = None):
        validate_request(prompt, steps or env.num_inference_steps)
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

    _routes(app, env, text2img, lambda n_inf: worker.submit_batched(n_inf, LOAD_PROMPT).result())
    return app


def _routes(app, env, text2img, run_load):
    @app.get("/")
    def read_main():
        return {"message": "This is" + env.model_id + " pod " + env.pod_name + " in AWS EC2 " + env.device +
                " instance; try /load/{n_runs}/infer/{n_inf}; /genimage http post with user prompt "}

    @app.get("/load/{n_runs}/infer/{n_inf}")
    def load(n_runs: int, n_inf: int):
        _check(LOAD_PROMPT, n_inf)
        t0 = time.time()
        report = benchmark(n_runs, "stable_diffusion_512", lambda: run_load(n_inf), env.pod_name)
        METRICS.request_done(env, time.time() - t0)
        return {"message": "benchmark report:" + report}

    @app.post("/genimage")
    def generate_image_post(request: dict):
        prompt = request.get("prompt")
        _check(prompt, env.num_inference_steps)
        img, latency = text2img(prompt)
        METRICS.request_done(env, float(latency))
        return {"prompt": prompt, "response": png_b64(img), "latency": latency}

    mount_ui(app, f"{env.model_id} on MI355X; pod {env.pod_name}", "/genimage", "{prompt: p}", output="image")


def _create_step_app(engine, env: ServerEnv, max_batch: int, title_suffix: str):
    from ..engines.diffusion import StepBatcher
    batcher = StepBatcher(engine, max_batch=max_batch)
    worker = StepBatchingWorker(batcher)

    # import-time warm-up (run-sd.py:144-146): capture every bucket's UNet-step graph (1, 2, 4, ... max_batch)
    # so no request pays a capture, then one short request end to end
    def warm():
        batcher.warmup()
    worker.call(warm)
    worker.submit(WARMUP_PROMPT, min(env.num_inference_steps, 2)).result()

    app = base_app(env, f"{env.model_id} SD2.1{title_suffix}", spaced=False)
    app.state.engine, app.state.worker, app.state.batcher = engine, worker, batcher

    def text2img(prompt: str, steps: Optional[int] = None):
        t0 = time.time()
        img = worker.submit(prompt, int(steps or env.num_inference_steps)).result()
        return img, str(time.time() - t0)

    _routes(app, env, text2img, lambda n_inf: worker.submit(LOAD_PROMPT, n_inf).result())
    return app


def main():
    run(create_app())


if __name__ == "__main__":
    main()
