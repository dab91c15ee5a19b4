"""Pre-sharded restart cache (weights.materialize shard_cache): a TP rank that
loaded a full HF checkpoint writes its own slice to tp{r}of{n}.safetensors, and a restarted
rank loads exactly the same tensors from that file without touching the checkpoint."""
import os

import pytest
import torch

from shai_amd.models.llama import LlamaConfig, LlamaForCausalLM
from shai_amd.parallel.state import TPState, set_tp, tp
from shai_amd.weights import materialize, shard_cache_path


@pytest.fixture
def hf_ckpt(tmp_path):
    transformers = pytest.importorskip("transformers")
    c = LlamaConfig.tiny()
    hc = transformers.LlamaConfig(vocab_size=c.vocab_size, hidden_size=c.hidden_size,
                                  intermediate_size=c.intermediate_size, num_hidden_layers=c.num_hidden_layers,
                                  num_attention_heads=c.num_attention_heads, num_key_value_heads=c.num_key_value_heads,
                                  head_dim=c.head_dim, rms_norm_eps=c.rms_norm_eps, rope_theta=c.rope_theta,
                                  max_position_embeddings=c.max_position_embeddings, tie_word_embeddings=False)
    torch.manual_seed(0)
    m = transformers.LlamaForCausalLM(hc).to(torch.bfloat16)
    d = tmp_path / "ckpt"
    m.save_pretrained(str(d), safe_serialization=True)
    return c, str(d)


@pytest.mark.parametrize("rank,size", [(0, 1), (1, 2)])
def test_shard_cache_roundtrip(hf_ckpt, tmp_path, rank, size):
    c, ckpt = hf_ckpt
    cache = str(tmp_path / "shards")
    saved = tp()
    set_tp(TPState(rank=rank, size=size))
    try:
        m1 = materialize(LlamaForCausalLM(c), "cpu", ckpt, shard_cache=cache)
        assert m1._shai_shard_cache == "written"
        path = shard_cache_path(cache, rank, size)
        assert os.path.isfile(path)
        # restarted worker: the checkpoint's tensors are never read again (corrupt it to prove it)
        for f in os.listdir(ckpt):
            if f.endswith(".safetensors"):
                with open(os.path.join(ckpt, f), "r+b") as fh:
                    fh.seek(100)
                    fh.write(b"\xff" * 64)
        m2 = materialize(LlamaForCausalLM(c), "cpu", ckpt, shard_cache=cache, seed=123)
        assert m2._shai_shard_cache == "hit"
        s1, s2 = m1.state_dict(), m2.state_dict()
        assert s1.keys() == s2.keys()
        for k in s1:
            assert torch.equal(s1[k], s2[k]), k
        # sharded: the fused QKV of rank r holds 1/size of the heads
        qkv = m2.model.layers[0].self_attn.qkv_proj.weight if hasattr(m2, "model") else None
        if qkv is not None:
            full = (c.num_attention_heads + 2 * c.num_key_value_heads) * c.head_dim
            assert qkv.shape[0] == full // size
    finally:
        set_tp(saved)


def test_shard_cache_layout_mismatch_is_rebuilt(hf_ckpt, tmp_path):
    c, ckpt = hf_ckpt
    cache = str(tmp_path / "shards")
    saved = tp()
    try:
        set_tp(TPState(rank=0, size=1))
        materialize(LlamaForCausalLM(c), "cpu", ckpt, shard_cache=cache)
        # a foreign file under this rank's name (different model layout) is ignored and rewritten
        os.replace(shard_cache_path(cache, 0, 1), shard_cache_path(cache, 0, 1) + ".bak")
        from safetensors.torch import save_file
        save_file({"x": torch.zeros(3)}, shard_cache_path(cache, 0, 1), metadata={"shai_class": "Other"})
        m = materialize(LlamaForCausalLM(c), "cpu", ckpt, shard_cache=cache)
        assert m._shai_shard_cache == "written"
    finally:
        set_tp(saved)
