"""Encoder model parity vs transformers reference implementations with identical
(bf16-representable) random weights, on the CPU fp32 path."""
import pytest
import torch

from shai_amd.weights import load_into

transformers = pytest.importorskip("transformers")


def _bf16_params(m):
    with torch.no_grad():
        for p in m.parameters():
            p.copy_(p.to(torch.bfloat16).float())
    return m.eval()


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-6)).item()


def test_distilbert_matches_transformers():
    from shai_amd.models.bert import DistilBertConfig, DistilBertForSequenceClassification
    c = DistilBertConfig.tiny()
    hc = transformers.DistilBertConfig(vocab_size=c.vocab_size, dim=c.dim, n_layers=c.n_layers, n_heads=c.n_heads,
                                       hidden_dim=c.hidden_dim, num_labels=2)
    torch.manual_seed(0)
    hf = _bf16_params(transformers.DistilBertForSequenceClassification(hc))
    m = DistilBertForSequenceClassification(c)
    load_into(m, {k: v.clone() for k, v in hf.state_dict().items()}, m.convert_hf_state_dict, strict=True)
    ids = torch.randint(0, 1000, (3, 12))
    mask = torch.ones(3, 12, dtype=torch.long)
    mask[1, 7:] = 0
    mask[2, 3:] = 0
    with torch.no_grad():
        ref = hf(input_ids=ids, attention_mask=mask).logits
        out = m(ids, mask)
    assert _rel(out, ref) < 0.03


def test_vit_matches_transformers():
    from shai_amd.models.vit import ViTConfig, ViTForImageClassification
    c = ViTConfig.tiny()
    hc = transformers.ViTConfig(image_size=64, patch_size=16, hidden_size=c.hidden_size,
                                num_hidden_layers=c.num_hidden_layers, num_attention_heads=c.num_attention_heads,
                                intermediate_size=c.intermediate_size, num_labels=c.num_labels)
    torch.manual_seed(1)
    hf = _bf16_params(transformers.ViTForImageClassification(hc))
    m = ViTForImageClassification(c)
    load_into(m, {k: v.clone() for k, v in hf.state_dict().items()}, m.convert_hf_state_dict, strict=True)
    px = torch.randn(2, 3, 64, 64).to(torch.bfloat16).float()
    with torch.no_grad():
        ref = hf(pixel_values=px).logits
        out = m(px.permute(0, 2, 3, 1).to(torch.bfloat16))
    assert _rel(out, ref) < 0.03


def test_t5_encoder_matches_transformers():
    from shai_amd.models.t5 import T5Config, T5EncoderModel
    c = T5Config.tiny()
    hc = transformers.T5Config(vocab_size=c.vocab_size, d_model=c.d_model, d_kv=c.d_kv, d_ff=c.d_ff,
                               num_layers=c.num_layers, num_heads=c.num_heads, feed_forward_proj="gated-gelu",
                               is_encoder_decoder=False, use_cache=False)
    torch.manual_seed(2)
    hf = _bf16_params(transformers.T5EncoderModel(hc))
    m = T5EncoderModel(c)
    load_into(m, {k: v.clone() for k, v in hf.state_dict().items()}, m.convert_hf_state_dict, strict=True)
    ids = torch.randint(2, 500, (2, 20))
    mask = torch.ones(2, 20, dtype=torch.long)
    mask[1, 13:] = 0
    with torch.no_grad():
        ref = hf(input_ids=ids, attention_mask=mask).last_hidden_state
        out = m(ids, mask)
    # compare valid positions (padded query rows are irrelevant to the API's consumers except the mean)
    assert _rel(out[0], ref[0]) < 0.03 and _rel(out[1, :13], ref[1, :13]) < 0.03


def test_yolos_matches_transformers():
    from shai_amd.models.vit import ViTConfig, YolosForObjectDetection
    c = ViTConfig.tiny(detection=True)
    hc = transformers.YolosConfig(image_size=[64, 64], patch_size=16, hidden_size=c.hidden_size,
                                  num_hidden_layers=c.num_hidden_layers, num_attention_heads=c.num_attention_heads,
                                  intermediate_size=c.intermediate_size, num_labels=c.num_labels,
                                  num_detection_tokens=c.num_detection_tokens, use_mid_position_embeddings=False)
    torch.manual_seed(3)
    hf = _bf16_params(transformers.YolosForObjectDetection(hc))
    m = YolosForObjectDetection(c)
    load_into(m, {k: v.clone() for k, v in hf.state_dict().items()}, m.convert_hf_state_dict, strict=True)
    px = torch.randn(1, 3, 64, 96).to(torch.bfloat16).float()   # non-native grid -> pos-embed interpolation
    with torch.no_grad():
        ref = hf(pixel_values=px)
        logits, boxes = m(px.permute(0, 2, 3, 1).to(torch.bfloat16))
    assert _rel(logits, ref.logits) < 0.05
    assert _rel(boxes, ref.pred_boxes) < 0.05
