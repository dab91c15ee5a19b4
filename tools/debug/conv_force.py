"""Per-case relative error of the forced-config conv cases of tests/test_gemm3_gpu.py (CONV_SCRIPT), plus the tuning
table entries used: run with SHAI_GEMM_FORCE=<cfg> set in the environment."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import shai_amd.ops as ops  # noqa: E402
from shai_amd.ops import reference as ref  # noqa: E402

torch.manual_seed(0)
cases = [(2, 32, 32, 64, 128, 3, 1, 1, False, 0), (2, 16, 16, 320, 320, 3, 1, 1, False, 0),
         (1, 16, 16, 64, 96, 3, 2, 1, False, 0), (2, 8, 8, 128, 64, 3, 1, 1, True, 0),
         (2, 16, 16, 96, 64, 3, 1, 1, False, 64), (2, 16, 16, 64, 64, 1, 1, 0, False, 0),
         (2, 32, 32, 320, 640, 3, 1, 1, False, 320), (2, 8, 8, 640, 320, 3, 1, 1, True, 640),
         (3, 12, 12, 128, 256, 3, 2, 1, False, 0),
         (20, 64, 64, 320, 320, 3, 1, 1, False, 0), (8, 48, 48, 128, 256, 3, 1, 1, True, 0)]
for N, H, C, Co, k, stride, pad, up, c2 in [(c[0], c[1], c[3], c[4], c[5], c[6], c[7], c[8], c[9]) for c in cases]:
    x = torch.randn(N, H, H, C, device="cuda").bfloat16()
    x2 = torch.randn(N, H, H, c2, device="cuda").bfloat16() if c2 else None
    cin = C + c2
    w = (torch.randn(Co, cin, k, k, device="cuda") / (cin * k * k) ** 0.5).bfloat16()
    wp = ops.pack_conv_weight(w)
    b = torch.randn(Co, device="cuda").bfloat16()
    y = ops.conv2d(x, wp, b, k, k, stride, pad, upsample=up, x2=x2, act="silu")
    yr = ref.conv2d(x.cpu(), wp.cpu(), b.cpu(), k, k, stride, pad, upsample=up,
                    x2=x2.cpu() if x2 is not None else None, act="silu")
    rel = ((y.float().cpu() - yr.float()).norm() / yr.float().norm()).item()
    print(N, H, C, Co, k, stride, pad, up, c2, "rel", round(rel, 5), flush=True)
for line in ops.gemm_tuning_table() if hasattr(ops, "gemm_tuning_table") else []:
    if line.startswith("1:") or line.startswith("2:"):
        print(line)
