"""T5 encoder embedding API, compatible with app/t5_model_api.py:
  POST /generate  {"prompt": str, "max_new_tokens": int}
       -> {"text": base64(str(np.ndarray mean-pooled embedding)), "execution_time": float}
       (input padded/truncated to max_length = max_new_tokens, mean over all positions)
  POST /benchmark {"n_runs", "max_new_tokens", "prompt"} -> {"report": base64(...)}
       (the reference passes 5 args to a 4-arg benchmark(), t5_model_api.py:64,139;
        the intended behaviour is implemented)
TP-sharded artifacts (tp_*.pt) are replaced by shard-on-load of the HF checkpoint:
``TENSOR_PARALLEL_SIZE=N`` runs the worker as N ranks (one GPU each); rank 0 broadcasts
each batched ``embed`` call to the others (serving/tp.py).
"""

import time
import traceback
from typing import Optional

import numpy as np

from .common import METRICS, EngineWorker, LatencyCollector, ServerEnv, b64text, base_app, latency_report


def build_engine(env: ServerEnv):
    from ..engines.encoders import TextEmbeddingEngine
    from ..models.t5 import T5Config
    m = env.model_id.lower()
    cfg = T5Config.tiny() if env.config == "tiny" else (T5Config.xxl() if "xxl" in m else T5Config.v1_1_large())
    return TextEmbeddingEngine(cfg, device=env.torch_device, model_path=env.model_path)


def _env():
    return ServerEnv.from_env(app="t5", model_id="google/t5-v1_1-large", max_seq_len=1024)


def create_app(engine=None, env: Optional[ServerEnv] = None, tpc=None):
    from fastapi import HTTPException
    from pydantic import BaseModel, Field
    env = env or _env()
    engine = engine or build_engine(env)
    if tpc is not None:
        engine = tpc.wrap(engine, ("embed",))
    worker = EngineWorker("t5", batch_fn=lambda L, args: list(engine.embed([a[0] for a in args], L)), max_batch=32,
                          max_wait_ms=2.0)

    class GenerateRequest(BaseModel):
        max_new_tokens: int
        prompt: str

    class GenerateBenchmarkRequest(BaseModel):
        n_runs: int
        max_new_tokens: int
        prompt: str

    class GenerateResponse(BaseModel):
        text: str = Field(..., description="Base64-encoded text")
        execution_time: float

    class GenerateBenchmarkResponse(BaseModel):
        report: str = Field(..., description="Benchmark report")

    def gentext(prompt, max_new_tokens):
        t0 = time.time()
        emb = worker.submit_batched(int(max_new_tokens), prompt).result()
        return str(np.asarray(emb, dtype=np.float32)), float(time.time() - t0)

    def bench(n_runs, test_name, prompt, max_new_tokens):
        lc = LatencyCollector()
        for _ in range(max(1, n_runs)):
            lc.pre_hook()
            gentext(prompt, max_new_tokens)
            lc.hook()
        return latency_report(lc, test_name)

    bench(2, "warmup", "What model are you?", env.max_seq_len)
    app = base_app(env, f"{env.model_id} embeddings", spaced=True)

    @app.post("/benchmark", response_model=GenerateBenchmarkResponse)
    def generate_benchmark_report(request: GenerateBenchmarkRequest):
        try:
            test_name = f"benchmark:{env.app} on {env.nodepool} with {request.max_new_tokens} output tokens"
            return GenerateBenchmarkResponse(report=b64text(bench(request.n_runs, test_name, request.prompt,
                                                                  request.max_new_tokens)))
        except Exception as e:
            traceback.print_exc()
            raise HTTPException(status_code=500, detail=f"{e}")

    @app.post("/generate", response_model=GenerateResponse)
    def generate_text_post(request: GenerateRequest):
        try:
            text, total = gentext(request.prompt, request.max_new_tokens)
            METRICS.request_done(env, total)
            return GenerateResponse(text=b64text(text), execution_time=total)
        except Exception as e:
            traceback.print_exc()
            raise HTTPException(status_code=500, detail=f"text serialization failed: {e}")

    return app


def main():
    from . import tp as tp_serving
    env = _env()
    tp_serving.serve("shai_amd.serving.t5_api", tp_serving.env_tp_degree(), lambda: build_engine(env),
                     lambda tpc: create_app(env=env, tpc=tpc))


if __name__ == "__main__":
    main()
