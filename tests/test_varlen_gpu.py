"""Packed varlen prefill on the GPU: the paged varlen flash-attention kernel vs an fp32 PyTorch reference for
sequences of 1 .. 8k new tokens over cached contexts, and the engine's packed prefill vs its padded path
(mixed prompt lengths 64 .. 8k)."""
import pytest
import torch

from shai_amd import ops
from shai_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("D", [64, 128])
def test_paged_attention_varlen_kernel(cuda, D):
    torch.manual_seed(0)
    Hq, Hkv = 8, 2
    n_cached = [0, 130, 0, 5000, 63]
    n_new = [64, 1, 8192, 700, 1]          # prefill chunks and decode rows in one packed step
    blocks_per = [(c + n + 63) // 64 for c, n in zip(n_cached, n_new)]
    nblk = sum(blocks_per) + 4
    kc = (torch.randn(nblk, Hkv, 64, D, device=cuda) * 0.5).bfloat16()
    vc = torch.randn(nblk, Hkv, 64, D, device=cuda).bfloat16()
    perm = torch.randperm(nblk).tolist()
    tables, o = [], 0
    for nb in blocks_per:
        tables.append(perm[o:o + nb])
        o += nb
    maxb = max(blocks_per)
    bt = torch.zeros(len(n_new), maxb, dtype=torch.int32)
    for i, t in enumerate(tables):
        bt[i, :len(t)] = torch.tensor(t)
    T = sum(n_new)
    q = torch.randn(T, Hq, D, device=cuda).bfloat16()
    q_start = torch.tensor([sum(n_new[:i]) for i in range(len(n_new))], dtype=torch.int32, device=cuda)
    kv_lens = torch.tensor([c + n for c, n in zip(n_cached, n_new)], dtype=torch.int32, device=cuda)
    q_lens = torch.tensor(n_new, dtype=torch.int32, device=cuda)
    bt = bt.to(cuda)
    got = ops.paged_attention_varlen(q, kc, vc, bt, kv_lens, q_lens, q_start, max(n_new))
    want = ref.paged_attention_varlen(q.float(), kc.float(), vc.float(), bt, kv_lens, q_lens, q_start,
                                      1.0 / D ** 0.5, True)
    for b in range(len(n_new)):
        s0, n = int(q_start[b]), n_new[b]
        a, w = got[s0:s0 + n].float(), want[s0:s0 + n]
        rel = ((a - w).norm() / w.norm()).item()
        assert rel < 2e-2, (b, rel)


def test_engine_packed_prefill_matches_padded(cuda):
    from shai_amd.engines.llm import LLMEngine, SamplingParams
    from shai_amd.models.llama import LlamaConfig
    c = LlamaConfig(vocab_size=2048, hidden_size=512, intermediate_size=1024, num_hidden_layers=2,
                    num_attention_heads=8, num_key_value_heads=2, head_dim=64, max_position_embeddings=16384)
    prompts = [[(7 * i) % 2000 + 3 for i in range(n)] for n in (64, 1000, 8000, 300)]
    p = SamplingParams(max_tokens=6, temperature=0.0, ignore_eos=True)

    def run(packed):
        e = LLMEngine(c, device="cuda:0", max_num_seqs=4, max_model_len=8192 + 64, enable_prefix_caching=False,
                      packed_prefill=packed, mixed_steps=False, prefill_token_budget=16384, seed=3)
        rec = []
        fwd = e.model.forward
        e.model.forward = lambda *a, **k: (lambda y: (rec.append(y.float().clone()), y)[1])(fwd(*a, **k))
        with torch.inference_mode():
            out = [s.output for s in e.generate(prompts, p)]
        return out, rec[0]
    want, l_pad = run(False)
    got, l_packed = run(True)
    rel = ((l_packed - l_pad).norm() / l_pad.norm()).item()
    assert rel < 2e-2, rel
    assert got == want
