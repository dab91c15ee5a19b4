"""What the SD2.1 ResNet conv epilogues cost: one 3x3 conv shape (batch-64 CFG rows) timed graph-replayed with
bias only, + per-image time embedding, + residual, + GroupNorm partials of the output (stats="gn"), and all of
them, on the tuned kernel.  python tools/bench_conv_epi.py [level ...]  (level 320 / 640 / 1280)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from shai_amd import ops  # noqa: E402
from tools.bench_kernels import graph_time  # noqa: E402


def main():
    levels = [int(x) for x in sys.argv[1:]] or [320, 640, 1280]
    with torch.inference_mode():
        for c in levels:
            hw = {320: 64, 640: 32, 1280: 16}[c]
            n = 64
            x = torch.randn(n, hw, hw, c, device="cuda").bfloat16()
            w = ops.pack_conv_weight((torch.randn(c, c, 3, 3, device="cuda") / (9 * c) ** 0.5).bfloat16())
            b = torch.randn(c, device="cuda").bfloat16()
            temb = torch.randn(n, c, device="cuda").bfloat16()
            res = torch.randn(n, hw, hw, c, device="cuda").bfloat16()
            flop = 2 * n * hw * hw * c * c * 9
            arms = {
                "bias": dict(),
                "+temb": dict(temb=temb),
                "+res": dict(residual=res),
                "+stats": dict(stats="gn"),
                "temb+stats": dict(temb=temb, stats="gn"),
                "res+stats": dict(residual=res, stats="gn"),
            }
            for name, kw in arms.items():
                t = graph_time(lambda: ops.conv2d(x, w, b, 3, 3, 1, 1, **kw), iters=8)
                print(f"conv {n}x{hw}x{hw}x{c} 3x3 {name:11s} {t * 1e6:8.1f} us  {flop / t / 1e12:6.0f} TF/s", flush=True)


if __name__ == "__main__":
    main()
