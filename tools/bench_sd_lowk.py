#!/usr/bin/env python3
"""SD2.1 batch-32 (CFG 64 images) level-1 low-K GEMMs: time, TF/s and HBM bytes/s of the tuned choice, with the
epilogue variants separated (GEGLU vs plain same-N vs plain half-N), to locate what bounds them.

python tools/bench_sd_lowk.py [--m 262144]
"""
import argparse
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

import shai_amd.ops as ops


def timeit(fn, iters=10, warmup=3):
    for _ in range(warmup):
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
    ap.add_argument("--m", type=int, default=262144)
    a = ap.parse_args()
    M = a.m
    rnd = lambda *s: (torch.randn(*s, device="cuda") * 0.5).bfloat16()
    rows = []
    with torch.inference_mode():
        for name, N, K, kw in [("geglu_up (glu gelu)", 2560, 320, dict(act="gelu", glu=True)),
                               ("plain N=2560", 2560, 320, {}),
                               ("plain N=1280", 1280, 320, {}),
                               ("qkv N=960", 960, 320, {}),
                               ("proj N=320 +res", 320, 320, dict(res=True)),
                               ("ff_down K=1280 +res", 320, 1280, dict(res=True))]:
            x, w = rnd(M, K), rnd(N, K) * (1 / math.sqrt(K))
            b = rnd(N)
            glu = kw.get("glu", False)
            nout = N // 2 if glu else N
            out = torch.empty(M, nout, device="cuda", dtype=torch.bfloat16)
            res = rnd(M, nout) if kw.get("res") else None
            if res is not None:
                fn = lambda: ops.gemm_into(x, w, res, b, residual=res)
            else:
                fn = lambda: ops.gemm_into(x, w, out, b, act=kw.get("act"), glu=glu)
            t = timeit(fn)
            fl = 2 * M * N * K
            by = M * K * 2 + N * K * 2 + M * nout * 2 * (2 if res is not None else 1)
            rows.append((name, M, N, K, t * 1e6, fl / t / 1e12, by / t / 1e12))
    print(f"{'gemm':24s} {'M':>7s} {'N':>5s} {'K':>5s} {'us':>8s} {'TF/s':>7s} {'TB/s':>6s}")
    for r in rows:
        print(f"{r[0]:24s} {r[1]:7d} {r[2]:5d} {r[3]:5d} {r[4]:8.1f} {r[5]:7.1f} {r[6]:6.2f}")
    for ln in ops.gemm_tuning_table() if hasattr(ops, "gemm_tuning_table") else []:
        if str(M) in ln:
            print(ln)


if __name__ == "__main__":
    main()
