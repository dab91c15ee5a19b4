"""Long-context serving benchmark (the reference's vLLM config: max_model_len 128000,
context_encoding_buckets [1024, 16384], continuous batching -- cova/mllama-32-11b-vllm-trn1-config.yaml:10-16).

Mistral-7B bf16 (random init) on one GPU: ``--background`` sequences are already decoding when a
``--prompt-len``-token prompt arrives; it is prefilled in ``--chunk``-token packed chunks that the
background decode rows join (mixed steps).  Reports the long prompt's TTFT and TPOT, the background
sequences' token rate DURING the long prefill (never zero with mixed steps), and the steady TPOT.

    python -m shai_amd.bench.long_context [--prompt-len 16384] [--chunk 8192] [--background 16] [--gen 128]
Prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import time

import numpy as np
import torch


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--prompt-len", type=int, default=16384)
    ap.add_argument("--chunk", type=int, default=8192)
    ap.add_argument("--background", type=int, default=16)
    ap.add_argument("--gen", type=int, default=128)
    ap.add_argument("--no-mix", action="store_true", help="alternate prefill chunks and decode steps instead")
    ap.add_argument("--model", default="mistral", choices=["mistral", "llama3_8b", "llama31_8b"],
                    help="llama31_8b: 128k context (64k / 128k lines: --prompt-len 65536 / 127744)")
    a = ap.parse_args(argv)
    from ..engines.llm import LLMEngine, SamplingParams
    from ..models.llama import LlamaConfig
    cfg = {"mistral": LlamaConfig.mistral_7b, "llama3_8b": LlamaConfig.llama3_8b,
           "llama31_8b": LlamaConfig.llama31_8b}[a.model]()
    P, G = a.prompt_len, a.gen
    if P + G + 64 > cfg.max_position_embeddings:
        raise SystemExit(f"{a.model}: prompt {P} + {G} generated exceeds its {cfg.max_position_embeddings} positions")
    eng = LLMEngine(cfg, device="cuda:0", max_num_seqs=a.background + 1, max_model_len=P + G + 64,
                    enable_prefix_caching=False, prefill_chunk=a.chunk, prefill_token_budget=max(a.chunk, 2048),
                    mixed_steps=not a.no_mix)
    rng = np.random.default_rng(0)
    params = SamplingParams(temperature=0.7, top_k=50, top_p=0.9, max_tokens=G, ignore_eos=True)
    def scenario():
        """background decoders streaming -> steady TPOT -> the long prompt arrives -> TTFT / TPOT"""
        bgs = [eng.add_request(rng.integers(10, cfg.vocab_size - 10, 128).tolist(),
                               SamplingParams(temperature=0.7, top_k=50, top_p=0.9, max_tokens=10 ** 6,
                                              ignore_eos=True))
               for _ in range(a.background)]
        while any(not s.output for s in bgs):
            eng.step()
        for _ in range(8):   # steady decode
            eng.step()
        torch.cuda.synchronize()
        n0, t0 = sum(len(s.output) for s in bgs), time.perf_counter()
        for _ in range(32):
            eng.step()
        torch.cuda.synchronize()
        steady = (time.perf_counter() - t0) / max(1, (sum(len(s.output) for s in bgs) - n0) / max(1, a.background))
        long = eng.add_request(rng.integers(10, cfg.vocab_size - 10, P).tolist(), params)
        bg0 = sum(len(s.output) for s in bgs)
        steps = 0
        while long.first_token_time is None:
            eng.step()
            steps += 1
        during = sum(len(s.output) for s in bgs) - bg0
        while not long.finished:
            eng.step()
        for s in bgs:   # retire the background sequences
            s.params.max_tokens = len(s.output) + 1
        while eng.has_work():
            eng.step()
        torch.cuda.synchronize()
        ttft = long.first_token_time - long.arrival
        tpot = (long.finish_time - long.first_token_time) / max(1, len(long.output) - 1)
        return ttft, tpot, steady, steps, during, len(long.output)

    with torch.inference_mode():
        eng.warmup_graphs()
        scenario()   # warm-up: GEMM tuning of this scenario's row counts, first-call costs
        ttft, tpot, steady_tpot, steps_prefill, bg_during, n_long = scenario()
    res = {"metric": f"{a.model} long-context: TTFT of a {P}-token prompt beside {a.background} decoding sequences",
           "model": cfg.__class__.__name__ + f"({a.model}, random init, bf16)", "prompt_len": P, "chunk": a.chunk,
           "background_seqs": a.background, "mixed_steps": not a.no_mix,
           "ttft_ms": round(1000 * ttft, 1), "prefill_tok_per_s": round(P / ttft, 1),
           "tpot_ms_long": round(1000 * tpot, 3), "steady_tpot_ms_background": round(1000 * steady_tpot, 3),
           "prefill_steps": steps_prefill, "background_tokens_during_prefill": int(bg_during),
           "gen_len": n_long}
    print(json.dumps(res), flush=True)
    return res


if __name__ == "__main__":
    main()
