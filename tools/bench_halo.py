"""Halo-tiled GroupNorm-fused conv vs the apply-pass path at the SD2.1 batch-32 (64-row CFG batch) UNet conv shapes.

For each shape: fused (halo kernel, 8 and 4 waves), the fallback (GroupNorm apply pass + tuned conv), and the bare
conv on a pre-normalised input (what the old path's conv alone cost).  Interleaved rounds in one process, median
of 20 timed launches each (csrc/kernels/conv_halo.hip; rule: A/B in one process)."""
import argparse
import json
import sys

import torch

sys.path.insert(0, ".")
from shai_amd import ops  # noqa: E402

SHAPES = [  # (N, H, W, C1, C2, Cout, temb, residual)
    (64, 64, 64, 320, 0, 320, True, False),
    (64, 64, 64, 320, 0, 320, False, True),
    (64, 64, 64, 320, 320, 320, True, False),
    (64, 64, 64, 640, 320, 320, True, False),
    (64, 32, 32, 320, 0, 640, True, False),
    (64, 32, 32, 640, 0, 640, False, True),
    (64, 32, 32, 640, 640, 640, True, False),
    (64, 32, 32, 1280, 640, 640, True, False),
    (64, 16, 16, 640, 0, 1280, True, False),
    (64, 16, 16, 1280, 0, 1280, False, True),
    (64, 16, 16, 1280, 1280, 1280, True, False),
    (64, 16, 16, 1280, 640, 1280, True, False),
]


PLAIN = [  # (N, H, W, C, Cout, upsample)
    (64, 32, 32, 640, 640, True),     # up block 2 -> 64x64 level
    (64, 16, 16, 1280, 1280, True),   # up block 1 -> 32x32 level
    (64, 64, 64, 320, 320, False),
    (64, 32, 32, 640, 640, False),
]


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * n)]
    for i in range(n):
        ev[2 * i].record()
        fn()
        ev[2 * i + 1].record()
    torch.cuda.synchronize()
    ts = sorted(ev[2 * i].elapsed_time(ev[2 * i + 1]) * 1e3 for i in range(n))
    return ts[n // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--shapes", type=int, default=len(SHAPES))
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    rows = []
    for (N, H, W, C1, C2, Co, te, re) in SHAPES[: args.shapes]:
        torch.manual_seed(0)
        x = torch.randn(N, H, W, C1, device=dev).bfloat16()
        x2 = torch.randn(N, H, W, C2, device=dev).bfloat16() if C2 else None
        cin = C1 + C2
        w = (torch.randn(Co, 9 * cin, device=dev) / (9 * cin) ** 0.5).bfloat16()
        b = torch.zeros(Co, device=dev).bfloat16()
        t = torch.randn(N, Co, device=dev).bfloat16() if te else None
        r = torch.randn(N, H, W, Co, device=dev).bfloat16() if re else None
        g = torch.ones(cin, device=dev).bfloat16()
        sc, sh = ops.groupnorm_stats(x, g, torch.zeros_like(g), 32, 1e-5, x2=x2)
        xn = ops.groupnorm_apply(x, sc, sh, True, x2=x2)

        def fused():
            return ops.conv2d(x, w, b, 3, 3, 1, 1, x2=x2, norm=(sc, sh, "silu"), temb=t, residual=r)

        def bare():
            return ops.conv2d(xn, w, b, 3, 3, 1, 1, temb=t, residual=r)

        res = {}
        ops.set_halo_conv(0, 0)
        bare()   # tune the plain conv once (its cache entry) before timing
        for _ in range(2):   # interleaved rounds
            ops.set_halo_conv(1, 8)
            res.setdefault("halo8", []).append(timeit(fused))
            ops.set_halo_conv(1, 4)
            res.setdefault("halo4", []).append(timeit(fused))
            ops.set_halo_conv(1, 9)
            res.setdefault("halo8sgb", []).append(timeit(fused))
            ops.set_halo_conv(0, 0)
            res.setdefault("apply+conv", []).append(timeit(fused))
            res.setdefault("conv", []).append(timeit(bare))
        flop = 2.0 * N * H * W * Co * 9 * cin
        row = {"shape": f"{N}x{H}x{W} {C1}+{C2}->{Co}" + (" temb" if te else "") + (" res" if re else ""),
               "gflop": round(flop / 1e9, 1)}
        for k, v in res.items():
            us = min(v)
            row[k + "_us"] = round(us, 1)
            row[k + "_tfs"] = round(flop / us / 1e6, 1)
        rows.append(row)
        print(json.dumps(row), flush=True)
    # plain 3x3 convs without a norm (upsample convs, conv2 of blocks whose input is not normalised): halo (mode 2)
    # vs the tuned conv (mode 0)
    for (N, H, W, C, Co, ups) in PLAIN[: args.shapes]:
        torch.manual_seed(1)
        x = torch.randn(N, H, W, C, device=dev).bfloat16()
        cin = C
        w = (torch.randn(Co, 9 * cin, device=dev) / (9 * cin) ** 0.5).bfloat16()
        b = torch.zeros(Co, device=dev).bfloat16()

        def plain():
            return ops.conv2d(x, w, b, 3, 3, 1, 1, upsample=ups)

        res = {}
        ops.set_halo_conv(0, 0)
        plain()
        for _ in range(2):
            ops.set_halo_conv(2, 8)
            res.setdefault("halo8", []).append(timeit(plain))
            ops.set_halo_conv(2, 4)
            res.setdefault("halo4", []).append(timeit(plain))
            ops.set_halo_conv(0, 0)
            res.setdefault("conv", []).append(timeit(plain))
        OH = 2 * H if ups else H
        flop = 2.0 * N * OH * OH * Co * 9 * cin
        row = {"shape": f"plain {N}x{H}x{W} {C}->{Co}" + (" up2x" if ups else ""), "gflop": round(flop / 1e9, 1)}
        for k, v in res.items():
            us = min(v)
            row[k + "_us"] = round(us, 1)
            row[k + "_tfs"] = round(flop / us / 1e6, 1)
        rows.append(row)
        print(json.dumps(row), flush=True)
    ops.set_halo_conv(1, 0)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
