import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import shai_amd.ops as ops
M, N, K = [int(v) for v in sys.argv[1:4]]
cfg = int(sys.argv[4]); mode = sys.argv[5]
a = torch.randn(M, K, device="cuda").bfloat16()
w = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
bias = torch.randn(N, device="cuda").bfloat16()
for _ in range(5):
    ops.gemm_into(a, w, out, bias if mode == "bias" else None, force_cfg=cfg)
torch.cuda.synchronize()
