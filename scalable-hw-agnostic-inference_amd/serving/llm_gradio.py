"""Causal-LM server compatible with app/run-llama.py (used for Llama-3-8B and
Mistral-7B, mistral/*-deploy.yaml run /run-llama.sh):

  GET  /                                  -> {"message": "This is<model> pod ..."}
  POST /gentext   {"prompt": str}         -> {"prompt", "response": str, "latency": str(seconds)}
  POST /sentiment {"prompt": str}         -> same, classification-prompted generation
  GET  /health, /readiness (no space: "<pod>is healthy"), /metrics, /serve

Generation: do_sample with temperature 0.7, top-k 50, top-p 0.9 and
MAX_NEW_TOKENS new tokens (run-llama.py:34-46), on the continuous-batching
engine (bf16; the reference's bitsandbytes 4-bit path is unnecessary with 288 GB).
"""

from typing import Optional

from .common import METRICS, ServerEnv, base_app, mount_ui, run
from .llm_api import build_service

SENTIMENT_TEMPLATE = "Classify the sentiment of the following text as positive, negative, or neutral:\n\n{}\n\nSentiment:"


def create_app(service=None, env: Optional[ServerEnv] = None):
    from pydantic import BaseModel

    from ..engines.llm import SamplingParams
    env = env or ServerEnv.from_env(app="llama", max_new_tokens=50)
    service = service or build_service(env)
    params = SamplingParams(temperature=0.7, top_k=50, top_p=0.9, max_tokens=env.max_new_tokens)

    def gentext(prompt):
        text, secs, _ = service.generate_text(prompt, params)
        return str(text), str(secs)

    def classify_sentiment(prompt):
        response, total = gentext(SENTIMENT_TEMPLATE.format(prompt))
        return response.split("Sentiment:")[-1].strip(), total

    gentext("write a poem")  # warm-up (run-llama.py:60)

    app = base_app(env, f"{env.model_id} text generation", spaced=False)

    class Item(BaseModel):
        prompt: str
        response: Optional[str] = None
        latency: Optional[str] = None

    @app.get("/")
    def read_main():
        return {"message": "This is" + env.model_id + " pod " + env.pod_name + " in AWS EC2 " + env.device +
                " instance; try /load/{n_runs}/infer/{n_inf}; /gentext http post with user prompt "}

    @app.post("/gentext")
    def generate_text_post(item: Item):
        item.response, item.latency = gentext(item.prompt)
        METRICS.request_done(env, float(item.latency))
        return {"prompt": item.prompt, "response": item.response, "latency": item.latency}

    @app.post("/sentiment")
    def classify_text_post(item: Item):
        item.response, item.latency = classify_sentiment(item.prompt)
        METRICS.request_done(env, float(item.latency))
        return {"prompt": item.prompt, "response": item.response, "latency": item.latency}

    mount_ui(app, f"{env.model_id} on MI355X; pod {env.pod_name}", "/gentext", "{prompt: p}")
    return app


def main():
    run(create_app())


if __name__ == "__main__":
    main()
