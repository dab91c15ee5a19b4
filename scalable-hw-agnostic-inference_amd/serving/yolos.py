"""YOLOS object-detection server, compatible with app/run-yolo.py (whose
/detectobj calls an undefined function, run-yolo.py:68 -- implemented here):
  POST /detectobj {"prompt": <image URL|path|data-URI|base64>}
       -> {"image": <prompt>, "response": [{"score", "label", "box": {xmin, ymin, xmax, ymax}}], "latency": float}
"""

import time
from typing import Optional

from .common import METRICS, EngineWorker, ServerEnv, base_app, mount_ui, run


def build_engine(env: ServerEnv):
    import os

    from ..engines.encoders import DetectorEngine
    from ..models.vit import ViTConfig
    cfg = ViTConfig.tiny(detection=True) if env.config == "tiny" else ViTConfig.yolos_tiny()
    edge = int(os.environ.get("YOLOS_SHORTEST_EDGE", "0")) or None
    return DetectorEngine(cfg, device=env.torch_device, model_path=env.model_path, shortest_edge=edge)


def create_app(engine=None, env: Optional[ServerEnv] = None):
    from pydantic import BaseModel

    from ..engines.encoders import load_image, synthetic_image
    env = env or ServerEnv.from_env(app="yolos", model_id="hustvl/yolos-tiny")
    engine = engine or build_engine(env)
    worker = EngineWorker("yolos", batch_fn=lambda key, args: engine.detect([a[0] for a in args]), max_batch=8,
                          max_wait_ms=2.0)

    def detect_obj_image(src):
        t0 = time.time()
        img = load_image(src) if isinstance(src, str) else src
        dets = worker.submit_batched(0, img).result()
        return dets, time.time() - t0

    detect_obj_image(synthetic_image())
    app = base_app(env, f"{env.compiled_model_id} object detection", spaced=False)

    class Item(BaseModel):
        prompt: str
        latency: float = 0.0

    @app.get("/")
    def read_main():
        return {"message": "This is" + env.compiled_model_id + " pod " + env.pod_name + " in AWS EC2 " + env.device +
                " instance; try /detectobj http post with image url; /serve "}

    @app.post("/detectobj")
    def detect_post(item: Item):
        dets, lat = detect_obj_image(item.prompt)
        METRICS.request_done(env, lat)
        return {"image": item.prompt, "response": dets, "latency": lat}

    mount_ui(app, f"{env.compiled_model_id}; pod {env.pod_name}", "/detectobj", "{prompt: p}")
    return app


def main():
    run(create_app())


if __name__ == "__main__":
    main()
