"""Llama-3.2-Vision on the GPU: the native path (MFMA GEMMs, flash attention with zero-padded heads, paged
cross-attention K/V, HIP-graph decode with cross layers) against the fp32 CPU reference model with the same
weights; full-size vision tower shape / finiteness."""
import numpy as np
import pytest
import torch

from shai_amd.engines.llm import LLMEngine, SamplingParams
from shai_amd.models.mllama import MllamaConfig, MllamaVisionModel, MllamaVisionConfig, preprocess_image

pytestmark = pytest.mark.gpu


def _img(h, w, seed=0):
    return (np.random.default_rng(seed).random((h, w, 3)) * 255).astype(np.uint8)


def test_mllama_tiny_gpu_matches_cpu():
    c = MllamaConfig.tiny()
    cpu = LLMEngine(c, device="cpu", max_num_seqs=4, max_model_len=256)
    gpu = LLMEngine(c, device="cuda", max_num_seqs=4, max_model_len=256)
    gpu.model.load_state_dict({k: v.to("cuda") for k, v in cpu.model.state_dict().items()})
    pre = preprocess_image(_img(40, 90), c.vision)
    with torch.inference_mode():
        a = cpu.model.encode_images(pre["pixel_values"][None], torch.tensor([pre["aspect_ratio_id"]]),
                                    [pre["num_tiles"]]).float()
        b = gpu.model.encode_images(pre["pixel_values"][None].cuda(), torch.tensor([pre["aspect_ratio_id"]]).cuda(),
                                    [pre["num_tiles"]]).float().cpu()
    assert torch.isfinite(b).all()
    assert (a - b).abs().max() / a.abs().max() < 5e-2
    p = SamplingParams(max_tokens=4, temperature=0.0, ignore_eos=True)
    with torch.inference_mode():
        oc = cpu.generate([[1, 33, 512, 17, 99, 250]], p)[0].output
        s = gpu.add_request([1, 33, 512, 17, 99, 250], p, image={**pre, "pixel_values": pre["pixel_values"].cuda()})
        t = gpu.add_request([1, 17, 99, 250, 7], p)          # text-only row in the same decode batch
        while not (s.finished and t.finished):
            gpu.step()
    assert s.output[0] == oc[0]
    assert len(t.output) == 4 and gpu.bm.num_free == gpu.num_kv_blocks
    assert any(k[1] for k in gpu._graphs)   # decode went through a captured graph with cross layers


def test_vision_tower_full_size_gpu():
    vc = MllamaVisionConfig()
    with torch.device("cuda"):
        m = MllamaVisionModel(vc)
    from shai_amd.models.layers import init_random_
    init_random_(m, 0)
    pre = preprocess_image(_img(700, 1000), vc, "cuda")
    assert pre["num_tiles"] == 4
    with torch.inference_mode():
        out = m(pre["pixel_values"][None], torch.tensor([pre["aspect_ratio_id"]], device="cuda"),
                [pre["num_tiles"]])
    assert out.shape == (1, 4 * 1601, 7680) and torch.isfinite(out.float()).all()
