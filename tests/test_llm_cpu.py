"""LLM engine on CPU (fp32 reference ops): HF transformers parity with the same
weights, paged-KV / prefix-cache / continuous-batching behaviour, native
block manager and scheduler helpers."""
import numpy as np
import pytest
import torch

from shai_amd.engines.llm import LLMEngine, SamplingParams, sample
from shai_amd.models.llama import LlamaConfig
from shai_amd.weights import load_into


def _hf_tiny():
    transformers = pytest.importorskip("transformers")
    c = LlamaConfig.tiny()
    hc = transformers.LlamaConfig(vocab_size=c.vocab_size, hidden_size=c.hidden_size,
                                  intermediate_size=c.intermediate_size, num_hidden_layers=c.num_hidden_layers,
                                  num_attention_heads=c.num_attention_heads, num_key_value_heads=c.num_key_value_heads,
                                  head_dim=c.head_dim, rms_norm_eps=c.rms_norm_eps, rope_theta=c.rope_theta,
                                  max_position_embeddings=c.max_position_embeddings, tie_word_embeddings=False)
    torch.manual_seed(0)
    m = transformers.LlamaForCausalLM(hc).eval()
    with torch.no_grad():
        for p in m.parameters():
            p.copy_(p.to(torch.bfloat16).float())  # bf16-representable weights
    return c, m


def test_llama_matches_transformers():
    c, hf = _hf_tiny()
    eng = LLMEngine(c, device="cpu", max_num_seqs=2, max_model_len=256, enable_prefix_caching=False)
    load_into(eng.model, {k: v.clone() for k, v in hf.state_dict().items()}, eng.model.convert_hf_state_dict,
              strict=True)
    prompt = [3, 17, 99, 250, 7, 7, 400, 12]
    with torch.no_grad():
        ref = hf(torch.tensor([prompt])).logits[0, -1].float()
    seq = eng.add_request(prompt, SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True))
    # capture the prefill logits through the model directly
    from shai_amd.runtime import build_prefill
    eng.step()
    assert seq.finished and seq.output[0] == int(ref.argmax())
    # greedy continuation equals HF greedy generate
    out = eng.generate([prompt], SamplingParams(max_tokens=6, temperature=0.0, ignore_eos=True))[0].output
    with torch.no_grad():
        g = hf.generate(torch.tensor([prompt]), max_new_tokens=6, do_sample=False)[0, len(prompt):].tolist()
    assert out[:3] == g[:3]


def test_continuous_batching_and_prefix_cache():
    eng = LLMEngine(LlamaConfig.tiny(), device="cpu", max_num_seqs=3, max_model_len=512)
    p = SamplingParams(max_tokens=4, temperature=0.0, ignore_eos=True)
    long = list(range(5, 205))
    a = eng.generate([long], p)[0].output
    hits0 = eng.stats["prefix_hit_tokens"]
    b = eng.generate([long], p)[0].output
    assert eng.stats["prefix_hit_tokens"] - hits0 == 192  # 3 full 64-token blocks reused
    assert a == b
    # more requests than max_num_seqs -> queued and completed
    outs = eng.generate([[i + 3, i + 9, 11] for i in range(7)], p)
    assert all(len(s.output) == 4 and s.finished for s in outs)
    assert eng.bm.num_free == eng.num_kv_blocks


def test_block_manager_native():
    from shai_amd.runtime import BlockManager, build_decode, build_prefill, sched_admit
    bm = BlockManager(8)
    a = bm.allocate(3)
    assert len(set(a)) == 3 and bm.num_free == 5
    bm.register(a[0], 123)
    bm.release(a)
    assert bm.num_free == 8
    got = bm.lookup_prefix([123, 456])
    assert got == [a[0]] and bm.refcount(a[0]) == 1
    with pytest.raises(MemoryError):
        bm.allocate(8)
    assert sched_admit([100, 100, 5000], free_blocks=10, running=0, max_seqs=8, token_budget=4096,
                       watermark_blocks=1) == 2
    pos, slots, lens, bt = build_decode([70, 3], [[4, 5], [9]], 4)
    assert pos.tolist() == [70, 3] and slots.tolist() == [5 * 64 + 6, 9 * 64 + 3] and lens.tolist() == [71, 4]
    pos, slots, lens, ql, bt, last = build_prefill([64, 0], [2, 3], [[1, 2], [3]], 3, 2)
    assert slots.tolist() == [2 * 64, 2 * 64 + 1, -1, 3 * 64, 3 * 64 + 1, 3 * 64 + 2]
    assert last.tolist() == [1, 5] and lens.tolist() == [66, 3]


def test_sampling():
    logits = torch.full((3, 100), -10.0)
    logits[:, 42] = 10.0
    logits[1, 7] = 9.0
    t = torch.tensor([0.0, 1.0, 0.7])
    out = sample(logits, t, torch.tensor([50, 1, 0]), torch.tensor([0.9, 0.9, 1.0]))
    assert out.tolist()[0] == 42 and out.tolist()[1] == 42


def test_chunked_prefill_matches_and_interleaves():
    """A 300-token prompt prefilled in 64-token chunks gives the same greedy tokens as one-shot prefill,
    and a sequence already decoding keeps producing tokens between the chunks."""
    c = LlamaConfig.tiny()
    p = SamplingParams(max_tokens=5, temperature=0.0, ignore_eos=True)
    long = [(7 * i) % 500 + 3 for i in range(300)]
    ref = LLMEngine(c, device="cpu", max_num_seqs=4, max_model_len=512, enable_prefix_caching=False)
    want = ref.generate([long], p)[0].output
    eng = LLMEngine(c, device="cpu", max_num_seqs=4, max_model_len=512, enable_prefix_caching=False,
                    prefill_chunk=64)
    short = eng.add_request([5, 6, 7], SamplingParams(max_tokens=40, temperature=0.0, ignore_eos=True))
    eng.step()                      # short prompt prefilled
    s = eng.add_request(long, p)
    lens = []
    while not s.finished:
        eng.step()
        lens.append(len(short.output))
    assert s.output == want
    # decode of the short sequence advanced while the long prompt was still being prefilled
    assert lens[4] > lens[0]
    assert eng.stats["prefill_tokens"] >= 300


def test_fp8_quantize_roundtrip_and_cpu_linear():
    """quantize_fp8_rows / dequant_fp8 on the host; ops.linear with w_scale equals the bf16 GEMM on
    the dequantised weight (the CPU path dequantises)."""
    from shai_amd import ops
    torch.manual_seed(0)
    w = torch.randn(64, 128) * 0.1
    w8, sc = ops.quantize_fp8_rows(w)
    wd = ops.dequant_fp8(w8, sc)
    assert w8.dtype == torch.float8_e4m3fn and wd.dtype == torch.bfloat16
    assert ((wd.float() - w).norm() / w.norm()).item() < 0.05
    x = torch.randn(3, 128).bfloat16()
    torch.testing.assert_close(ops.linear(x, w8, w_scale=sc), ops.linear(x, wd))


def test_fp8_engine_cpu_generates():
    c = LlamaConfig.tiny()
    eng = LLMEngine(c, device="cpu", max_num_seqs=2, max_model_len=128, enable_prefix_caching=False,
                    quantization="fp8")
    out = eng.generate([[1, 2, 3, 4]], SamplingParams(max_tokens=4, temperature=0.0, ignore_eos=True))[0].output
    assert len(out) == 4
    with pytest.raises(ValueError):
        LLMEngine(c, device="cpu", max_num_seqs=2, max_model_len=128, quantization="int3")


def test_async_lookahead_decode_matches_sync():
    """Decode steps enqueued one ahead of the host (device-side token feedback, look-ahead step past a stop
    token dropped) produce exactly the tokens of the synchronous engine: greedy with stop tokens that end
    sequences at different steps, and seeded top-k/top-p sampling; every KV block is returned."""
    c = LlamaConfig.tiny()
    prompts = [[3, 17, 99, 250, 7], [5, 6, 7], [400, 12, 13, 14, 15, 16], [9, 9]]
    mk = lambda a: LLMEngine(c, device="cpu", max_num_seqs=4, max_model_len=256, enable_prefix_caching=False,
                             seed=5, async_decode=a)
    g = SamplingParams(max_tokens=12, temperature=0.0, ignore_eos=True)
    ref = [s.output for s in mk(False).generate(prompts, g)]
    stops = [ref[0][4], ref[2][7]]  # end two sequences early, at different steps
    gs = SamplingParams(max_tokens=12, temperature=0.0, ignore_eos=True, stop_token_ids=stops)
    e_sync, e_async = mk(False), mk(True)
    want = [s.output for s in e_sync.generate(prompts, gs)]
    got_seqs = e_async.generate(prompts, gs)
    assert [s.output for s in got_seqs] == want
    assert any(len(o) < 12 for o in want)
    assert e_async._inflight is None and e_async.bm.num_free == e_async.num_kv_blocks
    sp = SamplingParams(max_tokens=10, temperature=0.8, top_k=20, top_p=0.9, ignore_eos=True)
    a = [s.output for s in mk(False).generate(prompts, sp)]
    b = [s.output for s in mk(True).generate(prompts, sp)]
    assert a == b and all(len(o) == 10 for o in a)
    # the async engine really ran ahead: decode steps were enqueued while a previous one was in flight
    e = mk(True)
    for p in prompts:
        e.add_request(p, g)
    ahead = 0
    while e.has_work():
        e.step()
        ahead += e._inflight is not None
    assert ahead >= 8


def test_packed_prefill_matches_padded_mixed_lengths():
    """Packed varlen prefill (no [B, S_max] padding rows) gives the padded path's logits and greedy tokens for
    prompts of very different lengths (3 .. 700 tokens) admitted together."""
    c = LlamaConfig.tiny()
    prompts = [[5, 6, 7], [(11 * i) % 500 + 3 for i in range(700)], [(3 * i) % 400 + 9 for i in range(64)],
               [(5 * i) % 300 + 1 for i in range(129)]]
    p = SamplingParams(max_tokens=6, temperature=0.0, ignore_eos=True)

    def run(packed):
        e = LLMEngine(c, device="cpu", max_num_seqs=4, max_model_len=1024, enable_prefix_caching=False,
                      packed_prefill=packed, mixed_steps=False)
        rec = []
        fwd = e.model.forward
        e.model.forward = lambda *a, **k: (lambda y: (rec.append(y.float().clone()), y)[1])(fwd(*a, **k))
        out = [s.output for s in e.generate(prompts, p)]
        return out, rec[0], e
    want, l_pad, _ = run(False)
    got, l_packed, e = run(True)
    assert got == want
    torch.testing.assert_close(l_packed, l_pad, rtol=2e-2, atol=2e-2)
    assert e.stats["prefill_tokens"] == sum(len(q) for q in prompts)   # real tokens, not B x S_max


def test_mixed_prefill_decode_steps():
    """Decode rows join packed prefill steps: a running sequence produces a token in EVERY step while a long
    prompt is prefilled in chunks (no alternation), and both sequences' greedy tokens equal the unmixed run."""
    c = LlamaConfig.tiny()
    long = [(7 * i) % 500 + 3 for i in range(300)]
    p_long = SamplingParams(max_tokens=5, temperature=0.0, ignore_eos=True)
    p_short = SamplingParams(max_tokens=30, temperature=0.0, ignore_eos=True)

    def run(mixed):
        e = LLMEngine(c, device="cpu", max_num_seqs=4, max_model_len=512, enable_prefix_caching=False,
                      prefill_chunk=64, mixed_steps=mixed, async_decode=False)
        short = e.add_request([5, 6, 7], p_short)
        e.step()
        s = e.add_request(long, p_long)
        per_step = []
        while not s.finished:
            n0 = len(short.output)
            e.step()
            per_step.append(len(short.output) - n0)
        while e.has_work():
            e.step()
        return short.output, s.output, per_step
    s_ref, l_ref, steps_ref = run(False)
    s_mix, l_mix, steps_mix = run(True)
    assert l_mix == l_ref and s_mix == s_ref
    assert all(d == 1 for d in steps_mix), steps_mix          # decoded in every step of the long prefill
    assert 0 in steps_ref                                      # the alternating engine stalls it


def test_sampled_async_matches_sync_with_stops_and_seeds():
    """temperature > 0 with stop tokens: the async engine's dropped look-ahead rows must not shift any other
    sequence's sampling noise (counter-based per-sequence uniforms), and SamplingParams.seed makes a request's
    tokens independent of its batch-mates."""
    c = LlamaConfig.tiny()
    prompts = [[3, 17, 99, 250, 7], [5, 6, 7], [400, 12, 13, 14, 15, 16], [9, 9]]
    mk = lambda a: LLMEngine(c, device="cpu", max_num_seqs=4, max_model_len=256, enable_prefix_caching=False,
                             seed=5, async_decode=a)
    sp = SamplingParams(max_tokens=12, temperature=0.9, top_k=30, top_p=0.95, ignore_eos=True)
    ref = [s.output for s in mk(False).generate(prompts, sp)]
    stops = [ref[0][3], ref[2][6]]
    sps = SamplingParams(max_tokens=12, temperature=0.9, top_k=30, top_p=0.95, ignore_eos=True, stop_token_ids=stops)
    want = [s.output for s in mk(False).generate(prompts, sps)]
    got = [s.output for s in mk(True).generate(prompts, sps)]
    assert got == want and any(len(o) < 12 for o in want)
    seeded = SamplingParams(max_tokens=8, temperature=1.0, top_k=0, top_p=1.0, ignore_eos=True, seed=1234)
    alone = mk(True).generate([prompts[1]], seeded)[0].output
    e = mk(True)
    together = e.generate([prompts[0], prompts[1], prompts[3]], seeded)
    assert together[1].output == alone


def test_decode_attention_rope_qkv_cpu_fallback_matches_two_step():
    """CPU path of ops.decode_attention_rope_qkv (the fused QKV-fold decode op) = linear with the folded RMSNorm
    followed by decode_attention_rope: same output, same KV-cache writes."""
    import torch
    from shai_amd import ops
    torch.manual_seed(0)
    B, K, H, Hk, D, nb = 3, 64, 4, 2, 16, 8
    x = torch.randn(B, K).bfloat16()
    w = (torch.randn((H + 2 * Hk) * D, K) / K ** 0.5).bfloat16()
    ang = torch.rand(256, D // 2) * 3
    cos, sin = ang.cos().contiguous(), ang.sin().contiguous()
    kc = torch.randn(nb, Hk, 64, D).bfloat16()
    vc = torch.randn(nb, Hk, 64, D).bfloat16()
    bt = torch.tensor([[0, 1], [2, 3], [4, 5]], dtype=torch.int32)
    lens = torch.tensor([5, 70, 1], dtype=torch.int32)
    pos = lens - 1
    slots = torch.stack([bt[b, (int(c) - 1) // 64] * 64 + (int(c) - 1) % 64 for b, c in enumerate(lens)]).int()
    kc2, vc2 = kc.clone(), vc.clone()
    o = ops.decode_attention_rope_qkv(x, w, 1e-5, kc, vc, bt, lens, pos, cos, sin, slots, H, Hk)
    qkv = ops.linear(x, w, rms_eps=1e-5)
    want = ops.decode_attention_rope(qkv, kc2, vc2, bt, lens, pos, cos, sin, slots, H, Hk)
    assert torch.equal(kc, kc2) and torch.equal(vc, vc2)
    assert torch.allclose(o.float(), want.float(), atol=1e-2, rtol=1e-2)
