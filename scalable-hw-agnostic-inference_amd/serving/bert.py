"""DistilBERT SST-2 sentiment server, compatible with app/run-bert.py:
  GET  /                           -> {"message": "This is<model> pod ..."}
  POST /sentiment {"prompt": str}  -> {"prompt", "response": "POSITIVE"|"NEGATIVE", "latency": float}
  GET  /health, /readiness ("<pod>is healthy"), /metrics, /serve; CORS "*".
DEVICE=cpu runs the fp32 CPU path (BASELINE.json config 1, the c7g "plumbing"
unit); otherwise the gfx950 kernels.  Concurrent requests are batched.
"""

import time
from typing import Optional

from .common import METRICS, EngineWorker, ServerEnv, base_app, mount_ui, run


def build_engine(env: ServerEnv):
    from ..engines.encoders import TextClassifierEngine
    from ..models.bert import DistilBertConfig
    cfg = DistilBertConfig.tiny() if env.config == "tiny" else DistilBertConfig()
    return TextClassifierEngine(cfg, device=env.torch_device, model_path=env.model_path)


def create_app(engine=None, env: Optional[ServerEnv] = None):
    from pydantic import BaseModel
    env = env or ServerEnv.from_env(app="bert", model_id="distilbert-base-uncased-finetuned-sst-2-english")
    engine = engine or build_engine(env)
    worker = EngineWorker("bert", batch_fn=lambda key, args: engine.classify([a[0] for a in args]), max_batch=64,
                          max_wait_ms=2.0)

    def classify_sentiment(prompt):
        t0 = time.time()
        label = worker.submit_batched(0, prompt).result()
        return label, time.time() - t0

    classify_sentiment("Hamilton is overrated and fails to live up to the hype as the best musical of past years.")
    app = base_app(env, f"{env.model_id} sentiment", spaced=False, cors=True)

    class Item(BaseModel):
        prompt: str
        response: Optional[str] = None
        latency: float = 0.0

    @app.get("/")
    def read_main():
        return {"message": "This is" + env.model_id + " pod " + env.pod_name + " in AWS EC2 " + env.device +
                " instance; try /load/{n_runs}/infer/{n_inf}; /gentext http post with user prompt "}

    @app.post("/sentiment")
    def classify_text_post(item: Item):
        item.response, item.latency = classify_sentiment(item.prompt)
        METRICS.request_done(env, item.latency)
        return {"prompt": item.prompt, "response": item.response, "latency": item.latency}

    mount_ui(app, f"{env.model_id}; pod {env.pod_name}", "/sentiment", "{prompt: p}")
    return app


def main():
    run(create_app())


if __name__ == "__main__":
    main()
