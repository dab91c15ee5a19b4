"""Llama-3.2-Vision (mllama) on CPU (fp32 reference ops) against transformers' MllamaForConditionalGeneration
with the same random weights: vision tower + projector states, image-conditioned and text-only greedy
generation through the LLM engine (paged cross-attention K/V), rows before <|image|>, preprocessing."""
import math

import numpy as np
import pytest
import torch

from shai_amd.engines.llm import LLMEngine, SamplingParams
from shai_amd.models.mllama import CLIP_MEAN, CLIP_STD, MllamaConfig, preprocess_image
from shai_amd.weights import load_into


def _hf_tiny():
    transformers = pytest.importorskip("transformers")
    c = MllamaConfig.tiny()
    t, v = c.text, c.vision
    hc = transformers.MllamaConfig(
        vision_config=dict(hidden_size=v.hidden_size, num_hidden_layers=v.num_hidden_layers,
                           num_global_layers=v.num_global_layers, attention_heads=v.attention_heads,
                           intermediate_size=v.intermediate_size, vision_output_dim=v.vision_output_dim,
                           image_size=v.image_size, patch_size=v.patch_size, max_num_tiles=v.max_num_tiles,
                           intermediate_layers_indices=list(v.intermediate_layers_indices)),
        text_config=dict(vocab_size=t.vocab_size, hidden_size=t.hidden_size, intermediate_size=t.intermediate_size,
                         num_hidden_layers=t.num_hidden_layers, num_attention_heads=t.num_attention_heads,
                         num_key_value_heads=t.num_key_value_heads, max_position_embeddings=t.max_position_embeddings,
                         cross_attention_layers=list(c.cross_attention_layers), bos_token_id=1, eos_token_id=2,
                         pad_token_id=0),
        image_token_index=c.image_token_index)
    torch.manual_seed(0)
    m = transformers.MllamaForConditionalGeneration(hc).eval()
    g = torch.Generator().manual_seed(1)
    with torch.no_grad():
        for name, p in m.named_parameters():
            if "gate" in name:
                p.copy_(torch.rand(p.shape, generator=g) * 0.7 + 0.3)
            elif p.dim() >= 2:
                fan = p[0].numel() if "embed" not in name else 1
                std = 1.0 / math.sqrt(fan) if "embed" not in name else 0.5
                p.copy_(torch.randn(p.shape, generator=g) * std)
            elif "norm" in name:
                p.copy_(1.0 + 0.1 * torch.randn(p.shape, generator=g))
            else:
                p.copy_(0.02 * torch.randn(p.shape, generator=g))
            p.copy_(p.to(torch.bfloat16).float())  # bf16-representable weights
    return c, m


def _engine(c, hf):
    eng = LLMEngine(c, device="cpu", max_num_seqs=4, max_model_len=256, enable_prefix_caching=True)
    load_into(eng.model, {k: v.clone() for k, v in hf.state_dict().items()}, eng.model.convert_hf_state_dict,
              strict=True)
    return eng


def _image(h=40, w=90, seed=0):
    return (np.random.default_rng(seed).random((h, w, 3)) * 255).astype(np.uint8)


def _hf_inputs(c, pre, prompt):
    px = pre["pixel_values"].float().permute(0, 3, 1, 2)[None, None]          # [1, 1, T, 3, S, S]
    nt = pre["num_tiles"]
    T = c.vision.max_num_tiles
    ar_mask = torch.zeros(1, 1, T, dtype=torch.long)
    ar_mask[..., :nt] = 1
    pos = prompt.index(c.image_token_index)
    cam = torch.zeros(1, len(prompt), 1, T, dtype=torch.long)
    cam[0, pos:, 0, :nt] = 1
    return dict(pixel_values=px, aspect_ratio_ids=torch.tensor([[pre["aspect_ratio_id"]]]),
                aspect_ratio_mask=ar_mask, cross_attention_mask=cam)


def test_preprocess_canvas_and_tiles():
    c = MllamaConfig.tiny()
    pre = preprocess_image(_image(40, 90), c.vision)
    assert pre["num_tiles"] == 2 and pre["pixel_values"].shape == (4, 56, 56, 3)
    assert pre["aspect_ratio_id"] == 2                     # (1 row, 2 cols) in [(1,1),(1,2),...]
    assert float(pre["pixel_values"][2:].abs().max()) == 0.0
    try:
        from transformers.models.mllama.image_processing_pil_mllama import MllamaImageProcessorPil
    except Exception:  # pragma: no cover - depends on the transformers build
        return
    proc = MllamaImageProcessorPil(size={"height": 56, "width": 56}, image_mean=list(CLIP_MEAN),
                                   image_std=list(CLIP_STD))
    from PIL import Image
    out = proc(images=[[Image.fromarray(_image(40, 90))]], return_tensors="pt")
    assert int(out["aspect_ratio_ids"][0, 0]) == pre["aspect_ratio_id"]
    ref = out["pixel_values"][0, 0].permute(0, 2, 3, 1)
    assert (ref - pre["pixel_values"].float()).abs().mean() < 0.05


def test_vision_tower_matches_transformers():
    c, hf = _hf_tiny()
    eng = _engine(c, hf)
    pre = preprocess_image(_image(), c.vision)
    inp = _hf_inputs(c, pre, [1, c.image_token_index])
    with torch.no_grad():
        vis = hf.model.vision_model(pixel_values=inp["pixel_values"], aspect_ratio_ids=inp["aspect_ratio_ids"],
                                    aspect_ratio_mask=inp["aspect_ratio_mask"]).last_hidden_state
        ref = hf.model.multi_modal_projector(vis).reshape(1, -1, c.text.hidden_size)
        ours = eng.model.encode_images(pre["pixel_values"][None], torch.tensor([pre["aspect_ratio_id"]]),
                                       [pre["num_tiles"]]).float()
    err = (ours - ref).abs().max() / ref.abs().max()
    assert err < 3e-2, float(err)


LONG = [1] + [(13 * i) % 400 + 20 for i in range(70)] + [512] + [(5 * i) % 400 + 20 for i in range(80)]


@pytest.mark.parametrize("prompt,chunk", [([1, 512, 17, 99, 250, 7], None),
                                          ([1, 33, 44, 512, 17, 99, 250, 7, 8], None),
                                          (LONG, 64)])    # chunked prefill; <|image|> in the 2nd chunk
def test_image_generation_matches_transformers(prompt, chunk):
    c, hf = _hf_tiny()
    eng = _engine(c, hf)
    eng.prefill_chunk = chunk or eng.prefill_chunk
    pre = preprocess_image(_image(), c.vision)
    inp = _hf_inputs(c, pre, prompt)
    with torch.no_grad():
        ref = hf(input_ids=torch.tensor([prompt]), **inp).logits[0, -1].float()
        g = hf.generate(input_ids=torch.tensor([prompt]), **inp, max_new_tokens=4, do_sample=False)
    s = eng.add_request(prompt, SamplingParams(max_tokens=4, temperature=0.0, ignore_eos=True), image=pre)
    while not s.finished:
        eng.step()
    assert s.output[0] == int(ref.argmax())
    assert s.output[:3] == g[0, len(prompt):len(prompt) + 3].tolist()
    assert eng.bm.num_free == eng.num_kv_blocks


def test_text_only_and_mixed_batch():
    c, hf = _hf_tiny()
    eng = _engine(c, hf)
    prompt = [1, 17, 99, 250, 7, 3]
    with torch.no_grad():
        g = hf.generate(input_ids=torch.tensor([prompt]), max_new_tokens=3, do_sample=False)[0, len(prompt):]
    p = SamplingParams(max_tokens=3, temperature=0.0, ignore_eos=True)
    a = eng.add_request(prompt, p)
    b = eng.add_request([1, 512, 5, 6], p, image=_image(70, 60, seed=3))   # same batch: image + text rows
    while not (a.finished and b.finished):
        eng.step()
    assert a.output == g.tolist()
    assert len(b.output) == 3 and eng.bm.num_free == eng.num_kv_blocks
    with pytest.raises(ValueError):
        LLMEngine(c.text, device="cpu", max_num_seqs=1, max_model_len=64).add_request([1, 2], p, image=_image())


def test_fp8_quantization_leaves_vision_tower_bf16():
    """``quantization: fp8`` converts the language model's TP linears only: every linear under the vision tower
    (no_fp8) keeps its bf16 weight (the tower's prefill-sized GEMMs must not silently go W8A8)."""
    from shai_amd.models.mllama import MllamaForConditionalGeneration
    from shai_amd.parallel.layers import FP8_LAYER_TYPES, quantize_fp8_
    torch.manual_seed(0)
    m = MllamaForConditionalGeneration(MllamaConfig.tiny())
    n = quantize_fp8_(m)
    assert n > 0
    vis = [mod for mod in m.vision_model.modules() if isinstance(mod, FP8_LAYER_TYPES)]
    txt = [mod for name, mod in m.named_modules()
           if isinstance(mod, FP8_LAYER_TYPES) and not name.startswith("vision_model")]
    assert vis and txt
    assert all(mod.weight.dtype == torch.bfloat16 for mod in vis)
    assert all(mod.weight.dtype == torch.float8_e4m3fn for mod in txt)
