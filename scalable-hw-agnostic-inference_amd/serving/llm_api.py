"""LLM JSON API -- compatible with app/vllm_model_api.py, app/vllm_model_api_m.py
(multimodal ``image`` field) and app/deepseek_model_api.py.

  POST /generate  {"prompt": str, "max_new_tokens": int, "image"?: base64}
                  -> {"text": base64(utf-8 text), "execution_time": float}
  POST /benchmark {"n_runs": int, "max_new_tokens": int, "prompt": str}
                  -> {"report": base64("RESULT FOR benchmark:<app> on <nodepool> with <n> output tokens: Latency P0=...")}
  GET  /health, /readiness ("<pod> is healthy"/"... is ready"), /metrics

Sampling defaults follow the reference (temperature 0.7, top-k 50, top-p 0.9,
app/vllm_model_api.py:24; ``SHAI_TEMPERATURE`` overrides the temperature, 0 =
greedy).  Unlike vllm_model_api.py:38-43, ``max_new_tokens`` is honoured (the _m
variant's behaviour).  Engine kwargs come from a /vllm_config.yaml-style file
(``VLLM_CONFIG``): tensor_parallel_size, max_num_seqs, max_model_len, block_size
(rounded to 64-token KV blocks), quantization (``fp8``: e4m3 weights + per-row
scales, bf16 activations).

Tensor parallelism (``tensor_parallel_size: N``, app/vllm_model_api.py:127-129 with
cova/mllama-32-11b-vllm-trn1-config.yaml:9): the worker runs as N processes, one
per GPU (the supervisor launches ``torch.distributed.run --nproc-per-node N``; a
bare ``python -m ...llm_api`` relaunches itself that way).  Rank 0 serves HTTP and
broadcasts each engine step's new requests to the other ranks, which run the same
step (serving/tp.py).

``image``: with a Llama-3.2-Vision model (``MODEL_ID`` containing "vision", or a
local checkpoint with a ``vision_config``) the image goes through the native
vision tower and the decoder's cross-attention layers (models/mllama.py); a
text-only model validates and acknowledges it without attending to it.
"""

import base64
import io
import os
import time
import traceback
from typing import Optional

from .common import METRICS, LatencyCollector, ServerEnv, b64text, base_app, latency_report, mount_ui


def load_vllm_config(path: Optional[str]) -> dict:
    if not path or not os.path.exists(path):
        return {}
    import yaml
    with open(path) as f:
        return yaml.safe_load(f) or {}


def _vllm_config() -> dict:
    return load_vllm_config(os.environ.get("VLLM_CONFIG", "/vllm_config.yaml"))


def tp_degree(vc: dict) -> int:
    from .tp import env_tp_degree
    return int(vc.get("tensor_parallel_size") or env_tp_degree())


def build_engine(env: ServerEnv, vc: Optional[dict] = None):
    """The (TP-sharded, when the process group is up) engine; identical on every rank."""
    from ..engines.llm import LLMEngine, llama_config_for
    vc = _vllm_config() if vc is None else vc
    cfg = llama_config_for(env.model_id, env.model_path, env.config)
    text = getattr(cfg, "text", cfg)   # MllamaConfig (vision) or LlamaConfig
    eng = LLMEngine(cfg, device=env.torch_device, model_path=env.model_path,
                    max_num_seqs=int(vc.get("max_num_seqs", 64)),
                    max_model_len=int(vc.get("max_model_len", min(8192, text.max_position_embeddings))),
                    enable_prefix_caching=True, quantization=vc.get("quantization"))
    import torch
    with torch.inference_mode():
        # every decode batch bucket (sampled and all-greedy) captured before the first request
        eng.warmup_graphs(greedy_too=True)
    return eng


def build_service(env: ServerEnv, tpc=None):
    from ..engines.llm import LLMService
    from ..tokenizers import load_tokenizer
    eng = build_engine(env)
    cfg = eng.mcfg if eng.mcfg is not None else eng.cfg
    text = eng.cfg
    specials = {"<|begin_of_text|>": text.bos_token_id}
    if text is not cfg:
        specials["<|image|>"] = cfg.image_token_index
    tok = load_tokenizer(env.model_path, vocab_size=text.vocab_size, bos_id=text.bos_token_id,
                         eos_id=text.eos_token_id, pad_id=0, model_max_length=eng.max_model_len, specials=specials)
    channel = None
    if tpc is not None and tpc.enabled:
        tpc.start_heartbeat()
        channel = tpc.channel
    return LLMService(eng, tok, channel=channel)


def _decode_image(b64: str):
    from PIL import Image
    raw = base64.b64decode(b64.split(",", 1)[-1])
    return Image.open(io.BytesIO(raw)).convert("RGB")


def add_instruct(prompt: str, has_image: bool) -> str:
    """Llama-3 instruct turn around the user prompt, with the image placeholder first when an image is
    attached (the formatting app/vllm_model_api_m.py:47 applies through NxDI's ``add_instruct``)."""
    img = "<|image|>" if has_image else ""
    return (f"<|begin_of_text|><|start_header_id|>user<|end_header_id|>\n\n{img}{prompt}<|eot_id|>"
            f"<|start_header_id|>assistant<|end_header_id|>\n\n")


def create_app(service=None, env: Optional[ServerEnv] = None, tpc=None):
    from fastapi import HTTPException
    from pydantic import BaseModel, Field

    from ..engines.llm import SamplingParams
    env = env or ServerEnv.from_env(app="llm")
    service = service or build_service(env, tpc)
    temperature = float(os.environ.get("SHAI_TEMPERATURE", "0.7"))

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
        return SamplingParams(temperature=temperature, top_k=50, top_p=0.9, max_tokens=max(1, int(n)))

    multimodal = bool(getattr(service, "multimodal", False))

    def gentext(prompt: str, max_new_tokens: int, image_b64: Optional[str] = None):
        image = None
        if image_b64:
            image = _decode_image(image_b64)
            prompt = add_instruct(prompt, True)
            if not multimodal:
                image = None  # text-only model: the image is validated and acknowledged, not attended to
        text, secs, _ = service.generate_text(prompt, params(max_new_tokens), image=image)
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
    from . import tp as tp_serving
    from ..engines.llm import engine_step
    vc = _vllm_config()
    env = ServerEnv.from_env(app="llm")
    # follower ranks mirror rank 0's engine steps (each STEP message = the requests admitted since the last)
    tp_serving.serve("shai_amd.serving.llm_api", tp_degree(vc), lambda: build_engine(env, vc),
                     lambda tpc: create_app(env=env, tpc=tpc),
                     step_fn=lambda eng: (lambda adds: engine_step(eng, adds)))


if __name__ == "__main__":
    main()
