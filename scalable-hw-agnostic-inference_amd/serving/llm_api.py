"""LLM JSON API -- compatible with app/vllm_model_api.py, app/vllm_model_api_m.py
(multimodal ``image`` field) and app/deepseek_model_api.py.

  POST /generate  {"prompt": str, "max_new_tokens": int, "image"?: base64}
                  -> {"text": base64(utf-8 text), "execution_time": float}
  POST /benchmark {"n_runs": int, "max_new_tokens": int, "prompt": str}
                  -> {"report": base64("RESULT FOR benchmark:<app> on <nodepool> with <n> output tokens: Latency P0=...")}
  GET  /health, /readiness ("<pod> is healthy"/"... is ready"), /metrics

Sampling defaults follow the reference (temperature 0.7, top-k 50, top-p 0.9,
app/vllm_model_api.py:24).  Unlike vllm_model_api.py:38-43, ``max_new_tokens``
is honoured (the _m variant's behaviour).  Engine kwargs can come from a
/vllm_config.yaml-style file (``VLLM_CONFIG``): tensor_parallel_size,
max_num_seqs, max_model_len, block_size (rounded to 64-token KV blocks).

``image``: decoded and validated; the Llama-3.2-Vision cross-attention tower is
not implemented, so the image is acknowledged but not attended to (see README).
"""

import base64
import io
import os
import time
import traceback
from typing import Optional

from .common import METRICS, LatencyCollector, ServerEnv, b64text, base_app, latency_report, mount_ui, run


def load_vllm_config(path: Optional[str]) -> dict:
    if not path or not os.path.exists(path):
        return {}
    import yaml
    with open(path) as f:
        return yaml.safe_load(f) or {}


def build_service(env: ServerEnv):
    from ..engines.llm import LLMEngine, LLMService, llama_config_for
    from ..tokenizers import load_tokenizer
    vc = load_vllm_config(os.environ.get("VLLM_CONFIG", "/vllm_config.yaml"))
    cfg = llama_config_for(env.model_id, env.model_path, env.config)
    eng = LLMEngine(cfg, device=env.torch_device, model_path=env.model_path,
                    max_num_seqs=int(vc.get("max_num_seqs", 64)),
                    max_model_len=int(vc.get("max_model_len", min(8192, cfg.max_position_embeddings))),
                    enable_prefix_caching=True)
    tok = load_tokenizer(env.model_path, vocab_size=cfg.vocab_size, bos_id=cfg.bos_token_id, eos_id=cfg.eos_token_id,
                         pad_id=0, model_max_length=eng.max_model_len)
    return LLMService(eng, tok)


def _decode_image(b64: str):
    from PIL import Image
    raw = base64.b64decode(b64.split(",", 1)[-1])
    return Image.open(io.BytesIO(raw)).convert("RGB")


def create_app(service=None, env: Optional[ServerEnv] = None):
    from fastapi import HTTPException
    from pydantic import BaseModel, Field

    from ..engines.llm import SamplingParams
    env = env or ServerEnv.from_env(app="llm")
    service = service or build_service(env)

    class GenerateRequest(BaseModel):
        max_new_tokens: int = 128
        prompt: str
        image: Optional[str] = None

    class GenerateBenchmarkRequest(BaseModel):
        n_runs: int
        max_new_tokens: int
        prompt: str

    class GenerateResponse(BaseModel):
        text: str = Field(..., description="Base64-encoded text")
        execution_time: float

    class GenerateBenchmarkResponse(BaseModel):
        report: str = Field(..., description="Benchmark report")

    def params(n):
        return SamplingParams(temperature=0.7, top_k=50, top_p=0.9, max_tokens=max(1, int(n)))

    def gentext(prompt: str, max_new_tokens: int, image_b64: Optional[str] = None):
        if image_b64:
            _decode_image(image_b64)  # validate; vision tower not implemented (see module doc)
            prompt = "<|image|>" + prompt
        text, secs, _ = service.generate_text(prompt, params(max_new_tokens))
        return text, secs

    def bench(n_runs, test_name, prompt, max_new_tokens):
        gentext(prompt, max_new_tokens)  # warm-up run, as the reference
        lc = LatencyCollector()
        for _ in range(max(1, n_runs)):
            lc.pre_hook()
            gentext(prompt, max_new_tokens)
            lc.hook()
        return latency_report(lc, test_name)

    # import-time warm-up (vllm_model_api.py:131-133 runs benchmark(10, "warmup"))
    bench(2, "warmup", "What model are you?", 8)

    app = base_app(env, f"{env.model_id} LLM API", spaced=True)
    app.state.service = service

    @app.post("/benchmark", response_model=GenerateBenchmarkResponse)
    def generate_benchmark_report(request: GenerateBenchmarkRequest):
        try:
            test_name = f"benchmark:{env.app} on {env.nodepool} with {request.max_new_tokens} output tokens"
            report = bench(request.n_runs, test_name, request.prompt, request.max_new_tokens)
            return GenerateBenchmarkResponse(report=b64text(report))
        except Exception as e:
            traceback.print_exc()
            raise HTTPException(status_code=500, detail=f"{e}")

    @app.post("/generate", response_model=GenerateResponse)
    def generate_text_post(request: GenerateRequest):
        try:
            text, total = gentext(request.prompt, request.max_new_tokens, request.image)
            METRICS.request_done(env, total)
            return GenerateResponse(text=b64text(text), execution_time=total)
        except Exception as e:
            traceback.print_exc()
            raise HTTPException(status_code=500, detail=f"text serialization failed: {e}")

    mount_ui(app, f"{env.model_id} on MI355X", "/generate", "{prompt: p, max_new_tokens: 64}")
    return app


def main():
    run(create_app())


if __name__ == "__main__":
    main()
