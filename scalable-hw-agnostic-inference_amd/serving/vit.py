"""ViT image-classification server, compatible with app/run-vit.py:
  GET  /                                 -> {"message": ...}
  POST /imgcls {"prompt": <image URL>}   -> {"image": <prompt>, "response": label, "latency": float}
``prompt`` may also be a file path, data-URI or raw base64 (the GPU box has no
network).  The model stays resident on the GPU (the reference reloads it per
request, run-vit.py:40-41) and concurrent requests are batched.
"""

import os
import time
from typing import Optional

from .common import METRICS, EngineWorker, ServerEnv, base_app, mount_ui, run


def build_engine(env: ServerEnv):
    from ..engines.encoders import ImageClassifierEngine
    from ..models.vit import ViTConfig
    cfg = ViTConfig.tiny() if env.config == "tiny" else ViTConfig.vit_base()
    return ImageClassifierEngine(cfg, device=env.torch_device, model_path=env.model_path)


def create_app(engine=None, env: Optional[ServerEnv] = None):
    from pydantic import BaseModel

    from ..engines.encoders import load_image, synthetic_image
    env = env or ServerEnv.from_env(app="vit", model_id="google/vit-base-patch16-224")
    engine = engine or build_engine(env)
    worker = EngineWorker("vit", batch_fn=lambda key, args: engine.classify([a[0] for a in args]), max_batch=32,
                          max_wait_ms=2.0)

    def classify_image(src):
        t0 = time.time()
        img = load_image(src) if isinstance(src, str) else src
        label = worker.submit_batched(0, img).result()
        return label, time.time() - t0

    classify_image(synthetic_image())  # warm-up (reference uses a COCO URL; no network here)
    if os.environ.get("SHAI_WARMUP_ALL_BATCHES", "1") != "0" and hasattr(engine, "warmup"):
        worker.call(lambda: engine.warmup(32))  # every batch size's graph, before the first request
    app = base_app(env, f"{env.compiled_model_id} image classification", spaced=False)

    class Item(BaseModel):
        prompt: str
        response: Optional[str] = None
        latency: float = 0.0

    @app.get("/")
    def read_main():
        return {"message": "This is" + env.compiled_model_id + " pod " + env.pod_name + " in AWS EC2 " + env.device +
                " instance; try /imgcls http post with image url; /serve "}

    @app.post("/imgcls")
    def classify_image_post(item: Item):
        item.response, item.latency = classify_image(item.prompt)
        METRICS.request_done(env, item.latency)
        return {"image": item.prompt, "response": item.response, "latency": item.latency}

    mount_ui(app, f"{env.compiled_model_id}; pod {env.pod_name}", "/imgcls", "{prompt: p}")
    return app


def main():
    run(create_app())


if __name__ == "__main__":
    main()
