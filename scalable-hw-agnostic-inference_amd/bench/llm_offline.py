"""Offline batched (multimodal) LLM latency harness -- counterpart of the reference's mllama-offline.py.

The reference (mllama-offline.py:54-113) runs 20 rounds of 4 (prompt, image-or-none, sampling) combos,
one request at a time through vLLM, and prints P0/50/90/95/99/100 latencies.  Here the same combos run
through the native engine (Llama-3.2-Vision or any text model: image combos are then sent text-only),
with synthetic images (the GPU box has no network for the reference's image URLs) and the reference's
percentile rule.  ``--concurrent`` submits each round's 4 requests together to exercise continuous
batching instead of bs=1.

    python -m shai_amd.bench.llm_offline --model meta-llama/Llama-3.2-11B-Vision-Instruct --rounds 20
"""
from __future__ import annotations

import argparse
import time

import numpy as np

PROMPTS = ["What is in this image? Tell me a story",
           "What is the recipe of mayonnaise in two sentences?",
           "Describe this image",
           "What is the capital of Italy famous for?"]
HAS_IMAGE = [True, False, True, False]
SAMPLING = [dict(top_k=1, temperature=1.0, top_p=1.0, max_tokens=256),
            dict(top_k=1, temperature=0.9, top_p=1.0, max_tokens=256),
            dict(top_k=10, temperature=0.9, top_p=0.5, max_tokens=512),
            dict(top_k=10, temperature=0.75, top_p=0.5, max_tokens=1024)]


def synthetic_images(seed: int = 0):
    rng = np.random.default_rng(seed)
    return [(rng.random((512, 768, 3)) * 255).astype(np.uint8), (rng.random((900, 1200, 3)) * 255).astype(np.uint8)]


def run(service, rounds: int = 20, concurrent: bool = False, max_tokens_cap: int = 0, log=print):
    """service: engines.llm.LLMService.  Returns the LatencyCollector."""
    from ..engines.llm import SamplingParams
    from ..serving.common import LatencyCollector, latency_report
    from ..serving.llm_api import add_instruct
    imgs = synthetic_images()
    mm = getattr(service, "multimodal", False)
    lc = LatencyCollector()
    for r in range(rounds):
        reqs = []
        for i, (p, has, sp) in enumerate(zip(PROMPTS, HAS_IMAGE, SAMPLING)):
            sp = dict(sp)
            if max_tokens_cap:
                sp["max_tokens"] = min(sp["max_tokens"], max_tokens_cap)
            params = SamplingParams(temperature=sp["temperature"], top_k=sp["top_k"], top_p=sp["top_p"],
                                    max_tokens=sp["max_tokens"])
            image = imgs[i // 2] if (has and mm) else None
            reqs.append((service.encode(add_instruct(p, image is not None)), params, image))
        if concurrent:
            t0 = time.perf_counter()
            futs = [service.submit_ids(ids, params, image) for ids, params, image in reqs]
            for f in futs:
                f.result()
            lc.latency_list.append(time.perf_counter() - t0)
        else:
            for ids, params, image in reqs:
                t0 = time.perf_counter()
                service.submit_ids(ids, params, image).result()
                lc.latency_list.append(time.perf_counter() - t0)
    log(latency_report(lc, "MLLAMA" if mm else "LLM"))
    return lc


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="meta-llama/Llama-3.2-11B-Vision-Instruct")
    ap.add_argument("--model-path", default=None)
    ap.add_argument("--config", default="", help="'tiny' for a smoke run")
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--concurrent", action="store_true")
    ap.add_argument("--max-tokens-cap", type=int, default=0)
    ap.add_argument("--device", default="cuda")
    a = ap.parse_args(argv)
    import torch
    from ..engines.llm import LLMEngine, LLMService, llama_config_for
    from ..tokenizers import load_tokenizer
    cfg = llama_config_for(a.model, a.model_path, a.config)
    text = getattr(cfg, "text", cfg)
    dev = a.device if torch.cuda.is_available() else "cpu"
    eng = LLMEngine(cfg, device=dev, model_path=a.model_path, max_num_seqs=8,
                    max_model_len=min(2048, text.max_position_embeddings))
    specials = {"<|begin_of_text|>": text.bos_token_id}
    if text is not cfg:
        specials["<|image|>"] = cfg.image_token_index
    tok = load_tokenizer(a.model_path, vocab_size=text.vocab_size, bos_id=text.bos_token_id,
                         eos_id=text.eos_token_id, model_max_length=eng.max_model_len, specials=specials)
    run(LLMService(eng, tok), a.rounds, a.concurrent, a.max_tokens_cap)


if __name__ == "__main__":
    main()
