#!/usr/bin/env python3
"""Per-shape timing of the SD2.1 UNet transformer GEMMs (batch 32 x CFG = 64 latents) for each GEMM
config vs hipBLASLt, with achieved TFLOP/s and HBM GB/s (A + W + C + residual bytes).

python tools/bench_sd_gemms.py [--cfgs 9,10] [--iters 20]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import shai_amd.ops as ops  # noqa: E402

# (M, N, K, glu, residual, bias)
SHAPES = [(262144, 320, 320, False, True, True), (262144, 2560, 320, True, False, True),
          (262144, 320, 1280, False, True, True), (262144, 960, 320, False, False, False),
          (65536, 640, 640, False, True, True), (65536, 5120, 640, True, False, True),
          (65536, 640, 2560, False, True, True), (65536, 1920, 640, False, False, False),
          (16384, 1280, 1280, False, True, True), (16384, 10240, 1280, True, False, True),
          (16384, 1280, 5120, False, True, True), (16384, 3840, 1280, False, False, False)]


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfgs", default="9,10")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    cfgs = [int(c) for c in a.cfgs.split(",") if c]
    dev = "cuda"
    print(f"{'shape':>28} {'cfg':>6} {'us':>8} {'TF/s':>7} {'GB/s':>7}")
    for M, N, K, glu, res, bias in SHAPES:
        x = torch.randn(M, K, device=dev).bfloat16()
        w = (torch.randn(N, K, device=dev) / K ** 0.5).bfloat16()
        b = torch.randn(N, device=dev).bfloat16() if bias else None
        nout = N // 2 if glu else N
        r = torch.randn(M, nout, device=dev).bfloat16() if res else None
        out = torch.empty(M, nout, device=dev, dtype=torch.bfloat16)
        flops = 2 * M * N * K
        byts = 2 * (M * K + N * K + M * nout + (M * nout if res else 0))
        tag = f"{M}x{N}x{K}{' glu' if glu else ''}{' +r' if res else ''}"
        runs = [(str(c), lambda c=c: ops.gemm_into(x, w, out, b, act="gelu" if glu else None, residual=r,
                                                     glu=glu, force_cfg=c)) for c in cfgs]
        runs.append(("tuned", lambda: ops.gemm_into(x, w, out, b, act="gelu" if glu else None, residual=r, glu=glu)))
        if not glu and not res:
            runs.append(("blas", lambda: torch.matmul(x, w.t(), out=out)))
        for name, fn in runs:
            try:
                t = timeit(fn, a.iters)
            except Exception as e:  # config unsupported for this shape
                print(f"{tag:>28} {name:>6} skipped: {e}")
                continue
            print(f"{tag:>28} {name:>6} {t * 1e6:8.1f} {flops / t / 1e12:7.0f} {byts / t / 1e9:7.0f}", flush=True)


if __name__ == "__main__":
    main()
