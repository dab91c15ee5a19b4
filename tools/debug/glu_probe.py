import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import shai_amd.ops as ops
from tools.bench_kernels import timeit
torch.manual_seed(0)
for (M, N, K) in [(65536, 2560, 320), (16384, 5120, 640), (8192, 8192, 8192)]:
    a = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    full = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    half = torch.empty(M, N // 2, device="cuda", dtype=torch.bfloat16)
    bias = torch.randn(N, device="cuda").bfloat16()
    for cfg in (1, 5, 6):
        r = {}
        r["plain"] = timeit(lambda: ops.gemm_into(a, w, full, force_cfg=cfg))
        r["bias"] = timeit(lambda: ops.gemm_into(a, w, full, bias, force_cfg=cfg))
        r["gelu"] = timeit(lambda: ops.gemm_into(a, w, full, act="gelu", force_cfg=cfg))
        r["glu_none"] = timeit(lambda: ops.gemm_into(a, w, half, act=None, glu=True, force_cfg=cfg))
        r["glu_gelu"] = timeit(lambda: ops.gemm_into(a, w, half, act="gelu", glu=True, force_cfg=cfg))
        print(f"{M}x{N}x{K} cfg{cfg} " + " ".join(f"{k}={v*1e6:.1f}us" for k, v in r.items()), flush=True)
    print(f"{M}x{N}x{K} torch {timeit(lambda: torch.matmul(a, w.t()))*1e6:.1f}us", flush=True)
