"""Debug: run skinny GPU tests one by one, then the tiny Llama engine with HF weights; report first NaN op."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch
import test_skinny_gpu as T
import test_models_gpu as MG
from shai_amd import ops
cuda = torch.device("cuda:0")
upto = sys.argv[1] if len(sys.argv) > 1 else "all"
tests = [("plain", lambda: [T.test_skinny_plain(cuda, *s) for s in [(1, 4096, 4096), (7, 6144, 4096), (32, 4096, 14336), (32, 28672, 4096), (16, 1024, 512), (32, 32768, 4096), (3, 96, 64)]]),
         ("glu", lambda: [T.test_skinny_glu_and_act(cuda, a) for a in ("silu", "gelu_tanh")]),
         ("graph", lambda: T.test_skinny_graph_replay_rearms_tickets(cuda)),
         ("auto", lambda: T.test_autotuned_decode_shapes(cuda)),
         ("folded", lambda: [T.test_folded_rmsnorm_linear(cuda, *s) for s in [(32, 6144, 4096), (5, 4096, 4096), (32, 28672, 4096), (64, 512, 1024)]]),
         ("rope", lambda: T.test_rope_qkv_cache(cuda))]
for name, fn in tests:
    if upto != "all" and name not in upto.split(","):
        continue
    fn(); torch.cuda.synchronize(); print("ran", name, flush=True)

def chk(name, t):
    torch.cuda.synchronize()
    bad = (~torch.isfinite(t.float())).sum().item()
    if bad:
        print(f"NONFINITE {name} shape={tuple(t.shape)} n={bad}", flush=True)
orig_linear = ops.linear
def lin(x, w, *a, **k):
    y = orig_linear(x, w, *a, **k); chk(f"linear M={x.shape[0]} N={w.shape[0]} K={w.shape[1]} rms={k.get('rms_eps')} glu={k.get('glu')}", y); return y
import shai_amd.parallel.layers as PL
PL.ops.linear = lin
try:
    MG.test_llama_engine_gpu_matches_transformers(cuda, False)
    print("engine test OK")
except Exception as e:
    print("engine test FAILED", type(e).__name__, str(e)[:200])
