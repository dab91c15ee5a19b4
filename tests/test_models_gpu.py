"""Model-level numerics on the MI355X: every model family runs through the HIP
kernels on cuda:0 and is compared against the transformers fp32 reference (same
bf16-representable random weights) or against our own CPU fp32 path."""
import numpy as np
import pytest
import torch

from shai_amd.weights import load_into

pytestmark = pytest.mark.gpu
transformers = pytest.importorskip("transformers")


def _bf16_params(m):
    with torch.no_grad():
        for p in m.parameters():
            p.copy_(p.to(torch.bfloat16).float())
    return m.eval()


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-6)).item()


def _hf_llama():
    from shai_amd.models.llama import LlamaConfig
    c = LlamaConfig.tiny()
    hc = transformers.LlamaConfig(vocab_size=c.vocab_size, hidden_size=c.hidden_size,
                                  intermediate_size=c.intermediate_size, num_hidden_layers=c.num_hidden_layers,
                                  num_attention_heads=c.num_attention_heads, num_key_value_heads=c.num_key_value_heads,
                                  head_dim=c.head_dim, rms_norm_eps=c.rms_norm_eps, rope_theta=c.rope_theta,
                                  max_position_embeddings=c.max_position_embeddings, tie_word_embeddings=False)
    torch.manual_seed(0)
    return c, _bf16_params(transformers.LlamaForCausalLM(hc))


@pytest.mark.parametrize("graphs", [False, True])
def test_llama_engine_gpu_matches_transformers(cuda, graphs):
    from shai_amd.engines.llm import LLMEngine, SamplingParams
    c, hf = _hf_llama()
    eng = LLMEngine(c, device="cuda", max_num_seqs=4, max_model_len=512, use_graphs=graphs)
    load_into(eng.model, {k: v.clone() for k, v in hf.state_dict().items()}, eng.model.convert_hf_state_dict,
              strict=True)
    prompts = [[3, 17, 99, 250, 7, 7, 400, 12], list(range(5, 140))]
    outs = eng.generate(prompts, SamplingParams(max_tokens=4, temperature=0.0, ignore_eos=True))
    for p, s in zip(prompts, outs):
        with torch.no_grad():
            g = hf.generate(torch.tensor([p]), max_new_tokens=4, do_sample=False)[0, len(p):].tolist()
        assert s.output[:2] == g[:2], (s.output, g)


def test_llm_engine_async_decode_gpu(cuda):
    """HIP-graph decode steps enqueued one ahead of the host (device-side token feedback, in-graph fused
    sampler, one pinned input copy per step) give exactly the synchronous engine's tokens: greedy with a
    stop token ending one sequence early (the batch stays in one graph bucket), and seeded sampling."""
    from shai_amd.engines.llm import LLMEngine, SamplingParams
    from shai_amd.models.llama import LlamaConfig
    c = LlamaConfig.tiny()
    prompts = [[3, 17, 99, 250, 7], [5, 6, 7], [400, 12, 13, 14, 15, 16], [9, 9]]
    mk = lambda a: LLMEngine(c, device="cuda", max_num_seqs=4, max_model_len=256, enable_prefix_caching=False,
                             seed=3, async_decode=a)
    g = SamplingParams(max_tokens=12, temperature=0.0, ignore_eos=True)
    ref = [s.output for s in mk(False).generate(prompts, g)]
    # a stop token that ends exactly one sequence, after its 4th token (so the batch stays in one bucket)
    cand = [(j, i, t) for j, o in enumerate(ref) for i, t in enumerate(o)
            if i >= 3 and t not in o[:i] and all(t not in q for k, q in enumerate(ref) if k != j)]
    if not cand:
        pytest.skip("no token unique to one sequence in this random model's greedy outputs")
    j, i, t = cand[0]
    gs = SamplingParams(max_tokens=12, temperature=0.0, ignore_eos=True, stop_token_ids=[t])
    want = [s.output for s in mk(False).generate(prompts, gs)]
    e = mk(True)
    with torch.inference_mode():
        assert e.warmup_graphs(greedy_too=True) == 6   # buckets 1, 2, 4 x {sampled, greedy}
    got = [s.output for s in e.generate(prompts, gs)]
    assert got == want and len(want[j]) == i + 1
    assert e._inflight is None and e.bm.num_free == e.num_kv_blocks
    sp = SamplingParams(max_tokens=16, temperature=0.8, top_k=40, top_p=0.9, ignore_eos=True)
    a = [s.output for s in mk(False).generate(prompts, sp)]
    b = [s.output for s in mk(True).generate(prompts, sp)]
    assert a == b and all(len(o) == 16 for o in a)


def test_llama_prefill_logits_gpu(cuda):
    """Full-sequence logits of the paged prefill path vs HF (bf16 tolerance)."""
    from shai_amd.models.llama import Batch
    from shai_amd.engines.llm import LLMEngine
    from shai_amd.runtime import build_prefill
    c, hf = _hf_llama()
    eng = LLMEngine(c, device="cuda", max_num_seqs=2, max_model_len=512, use_graphs=False)
    load_into(eng.model, {k: v.clone() for k, v in hf.state_dict().items()}, eng.model.convert_hf_state_dict,
              strict=True)
    ids = list(range(7, 7 + 100))
    with torch.no_grad():
        ref = hf(torch.tensor([ids])).logits[0, -1]
    from shai_amd.engines.llm import SamplingParams
    s = eng.add_request(ids, SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True))
    eng.step()
    assert s.output[0] == int(ref.argmax())


def test_encoders_gpu_match_transformers(cuda):
    from shai_amd.models.bert import DistilBertConfig, DistilBertForSequenceClassification
    from shai_amd.models.t5 import T5Config, T5EncoderModel
    from shai_amd.models.vit import ViTConfig, ViTForImageClassification, YolosForObjectDetection
    dev = torch.device("cuda")
    # DistilBERT
    c = DistilBertConfig.tiny()
    torch.manual_seed(0)
    hf = _bf16_params(transformers.DistilBertForSequenceClassification(transformers.DistilBertConfig(
        vocab_size=c.vocab_size, dim=c.dim, n_layers=c.n_layers, n_heads=c.n_heads, hidden_dim=c.hidden_dim,
        num_labels=2)))
    m = DistilBertForSequenceClassification(c)
    load_into(m, {k: v.clone() for k, v in hf.state_dict().items()}, m.convert_hf_state_dict, strict=True)
    m.to(dev)
    ids = torch.randint(0, 1000, (3, 12))
    mask = torch.ones(3, 12, dtype=torch.long)
    mask[1, 7:] = 0
    with torch.no_grad():
        assert _rel(m(ids.to(dev), mask.to(dev)), hf(input_ids=ids, attention_mask=mask).logits) < 0.05
    # ViT
    c = ViTConfig.tiny()
    torch.manual_seed(1)
    hf = _bf16_params(transformers.ViTForImageClassification(transformers.ViTConfig(
        image_size=64, patch_size=16, hidden_size=c.hidden_size, num_hidden_layers=c.num_hidden_layers,
        num_attention_heads=c.num_attention_heads, intermediate_size=c.intermediate_size, num_labels=c.num_labels)))
    m = ViTForImageClassification(c)
    load_into(m, {k: v.clone() for k, v in hf.state_dict().items()}, m.convert_hf_state_dict, strict=True)
    m.to(dev)
    px = torch.randn(2, 3, 64, 64).to(torch.bfloat16).float()
    with torch.no_grad():
        assert _rel(m(px.permute(0, 2, 3, 1).to(torch.bfloat16).to(dev)), hf(pixel_values=px).logits) < 0.05
    # YOLOS (interpolated position embeddings)
    c = ViTConfig.tiny(detection=True)
    torch.manual_seed(3)
    hf = _bf16_params(transformers.YolosForObjectDetection(transformers.YolosConfig(
        image_size=[64, 64], patch_size=16, hidden_size=c.hidden_size, num_hidden_layers=c.num_hidden_layers,
        num_attention_heads=c.num_attention_heads, intermediate_size=c.intermediate_size, num_labels=c.num_labels,
        num_detection_tokens=c.num_detection_tokens, use_mid_position_embeddings=False)))
    m = YolosForObjectDetection(c)
    load_into(m, {k: v.clone() for k, v in hf.state_dict().items()}, m.convert_hf_state_dict, strict=True)
    m.to(dev)
    px = torch.randn(1, 3, 64, 96).to(torch.bfloat16).float()
    with torch.no_grad():
        ref = hf(pixel_values=px)
        logits, boxes = m(px.permute(0, 2, 3, 1).to(torch.bfloat16).to(dev))
    assert _rel(logits, ref.logits) < 0.08 and _rel(boxes, ref.pred_boxes) < 0.08
    # T5 encoder
    c = T5Config.tiny()
    torch.manual_seed(2)
    hf = _bf16_params(transformers.T5EncoderModel(transformers.T5Config(
        vocab_size=c.vocab_size, d_model=c.d_model, d_kv=c.d_kv, d_ff=c.d_ff, num_layers=c.num_layers,
        num_heads=c.num_heads, feed_forward_proj="gated-gelu", is_encoder_decoder=False, use_cache=False)))
    m = T5EncoderModel(c)
    load_into(m, {k: v.clone() for k, v in hf.state_dict().items()}, m.convert_hf_state_dict, strict=True)
    m.to(dev)
    ids = torch.randint(2, 500, (2, 20))
    mask = torch.ones(2, 20, dtype=torch.long)
    mask[1, 13:] = 0
    with torch.no_grad():
        ref = hf(input_ids=ids, attention_mask=mask).last_hidden_state
        out = m(ids.to(dev), mask.to(dev))
    assert _rel(out[0], ref[0]) < 0.05 and _rel(out[1, :13], ref[1, :13]) < 0.05


def test_encoder_engines_gpu(cuda):
    """Engine-level entry points used by the servers (random-init production configs)."""
    from shai_amd.engines.encoders import (DetectorEngine, ImageClassifierEngine, TextClassifierEngine,
                                           TextEmbeddingEngine, synthetic_image)
    from shai_amd.models.t5 import T5Config
    tc = TextClassifierEngine()
    r = tc.classify(["I love this", "terrible"])
    assert len(r) == 2 and all(isinstance(x, str) for x in r)
    ic = ImageClassifierEngine()
    img = synthetic_image(480, 640)
    assert isinstance(ic.classify([img])[0], str)
    det = DetectorEngine()
    assert isinstance(det.detect([img])[0], list)
    te = TextEmbeddingEngine(cfg=T5Config.tiny())
    e = te.embed(["hello world"], 32)
    assert e.shape[-1] == T5Config.tiny().d_model and np.isfinite(e).all()


def test_vit_graph_replay_matches_eager(cuda):
    """The classifier's captured HIP graph gives the eager forward's logits, across replays with new inputs."""
    from shai_amd.engines.encoders import ImageClassifierEngine
    from shai_amd.models.vit import ViTConfig
    eng = ImageClassifierEngine(ViTConfig.vit_base(), device=cuda, seed=0)
    for i in range(3):
        x = torch.randint(0, 256, (4, 224, 224, 3), device=cuda, dtype=torch.uint8)
        got = eng.logits_u8(x).float().clone()
        want = eng._forward_u8(x).float()
        assert torch.allclose(got, want, atol=1e-2, rtol=1e-2), i


def test_vit_warmup_captures_every_batch(cuda):
    """A serving replica captures every batch size's graph up front; a later batch replays it."""
    from shai_amd.engines.encoders import ImageClassifierEngine
    from shai_amd.models.vit import ViTConfig
    eng = ImageClassifierEngine(ViTConfig.vit_base(), device=cuda, seed=0)
    assert eng.warmup(5) == 5
    x = torch.randint(0, 256, (3, 224, 224, 3), device=cuda, dtype=torch.uint8)
    got = eng.logits_u8(x).float().clone()
    assert len(eng._graphs) == 5
    assert torch.allclose(got, eng._forward_u8(x).float(), atol=1e-2, rtol=1e-2)


def test_async_decode_batch_shrinks_across_buckets_without_warmup(cuda):
    """Sequences of different lengths finish at different steps, so the running batch shrinks 4 -> 2 -> 1
    across graph buckets; nothing is pre-captured, so the async engine captures new buckets (and flips between
    sampled and all-greedy graphs) while a look-ahead step is in flight.  Tokens must equal the sync engine's."""
    from shai_amd.engines.llm import LLMEngine, SamplingParams
    from shai_amd.models.llama import LlamaConfig
    c = LlamaConfig.tiny()
    prompts = [[3, 17, 99, 250, 7], [5, 6, 7], [400, 12, 13, 14, 15, 16], [9, 9]]
    mk = lambda a: LLMEngine(c, device="cuda", max_num_seqs=4, max_model_len=256, enable_prefix_caching=False,
                             seed=11, async_decode=a)
    params = [SamplingParams(max_tokens=n, temperature=t, top_k=40, top_p=0.9, ignore_eos=True)
              for n, t in ((3, 0.8), (6, 0.0), (9, 0.0), (14, 0.0))]

    def run(e):
        with torch.inference_mode():
            seqs = [e.add_request(p, sp) for p, sp in zip(prompts, params)]
            while e.has_work():
                e.step()
        return [s.output for s in seqs], e
    want, _ = run(mk(False))
    got, e = run(mk(True))
    assert got == want and [len(o) for o in got] == [3, 6, 9, 14]
    assert {k[0] for k in e._graphs} >= {1, 2, 4}          # three buckets captured on the fly
    assert e._inflight is None and e.bm.num_free == e.num_kv_blocks


def test_decode_splits_grow_with_long_context(cuda):
    """A long-context sequence among many short ones raises the decode split-K factor (one graph per split
    count); tokens match the eager engine."""
    from shai_amd.engines.llm import LLMEngine, SamplingParams
    from shai_amd.models.llama import LlamaConfig
    c = LlamaConfig(vocab_size=1024, hidden_size=512, intermediate_size=512, num_hidden_layers=2,
                    num_attention_heads=8, num_key_value_heads=8, head_dim=64, max_position_embeddings=8192)
    mk = lambda g: LLMEngine(c, device="cuda", max_num_seqs=32, max_model_len=6000, enable_prefix_caching=False,
                             seed=2, use_graphs=g)
    e = mk(True)
    assert e.decode_splits(32, 100) < e.decode_splits(32, 5000)
    prompts = [[(5 * i) % 1000 + 3 for i in range(5000)]] + [[1 + j, 2, 3 + j] for j in range(20)]
    sp = SamplingParams(max_tokens=5, temperature=0.0, ignore_eos=True)
    with torch.inference_mode():
        got = [s.output for s in e.generate(prompts, sp)]
        want = [s.output for s in mk(False).generate(prompts, sp)]
    assert got == want
    assert any(k[0] == 32 and k[3] > e.decode_splits(32, 0) for k in e._graphs)
