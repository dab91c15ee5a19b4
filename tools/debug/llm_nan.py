"""Debug: locate NaNs in the tiny Llama GPU path (prefill + decode) vs the CPU reference."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from shai_amd.engines.llm import LLMEngine, SamplingParams
from shai_amd.models.llama import LlamaConfig
from shai_amd import ops

c = LlamaConfig.tiny()
torch.manual_seed(0)
eng = LLMEngine(c, device="cuda", max_num_seqs=4, max_model_len=512, use_graphs=False)
m = eng.model
# per-op NaN checks
orig_linear = ops.linear
def chk(name, t):
    torch.cuda.synchronize()
    bad = (~torch.isfinite(t.float())).sum().item()
    print(f"{name:30s} shape={tuple(t.shape)} nonfinite={bad} absmax={t.float().abs().max().item():.3g}", flush=True)
def lin(x, w, *a, **k):
    y = orig_linear(x, w, *a, **k)
    chk(f"linear N={w.shape[0]} K={w.shape[1]} rms={k.get('rms_eps')}", y)
    return y
ops.linear = lin
import shai_amd.parallel.layers as PL
PL.ops.linear = lin
orig_rq = ops.rope_qkv_cache
def rq(qkv, *a, **k):
    r = orig_rq(qkv, *a, **k)
    chk("rope_qkv_cache qkv", qkv)
    return r
ops.rope_qkv_cache = rq
import shai_amd.models.llama as L
L.ops.rope_qkv_cache = rq
orig_da = ops.decode_attention
def da(*a, **k):
    o = orig_da(*a, **k); chk("decode_attention", o); return o
L.ops.decode_attention = da
orig_pa = ops.paged_attention
def pa(*a, **k):
    o = orig_pa(*a, **k); chk("paged_attention", o); return o
L.ops.paged_attention = pa
prompts = [[3, 17, 99, 250, 7, 7, 400, 12], list(range(5, 140))]
outs = eng.generate(prompts, SamplingParams(max_tokens=3, temperature=0.0, ignore_eos=True))
print([s.output for s in outs])
